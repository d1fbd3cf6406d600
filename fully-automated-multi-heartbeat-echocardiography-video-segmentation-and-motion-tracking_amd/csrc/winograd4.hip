// Fused Winograd F(4x4, 3x3) for the stride-1 1x3x3 fp32 convs (R(2+1)D-18 Conv2Plus1D spatial halves:
// 56x56, 28x28, 14x14 and 7x7 maps at 112x112 clips -- the last two with partial edge tiles;
// torchvision Conv2Plus1D's first conv, called through src/model/R2plus1D_18_MotionNet.py:31-37).
//
// Arithmetic: Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A with Lavin's F(4,3) matrices (points 0, +-1,
// +-2): 36 Winograd-domain products per 4x4 outputs and channel pair instead of conv_wino_q's 64 (F(2x2,
// 3x3), 16 per 2x2) -- 0.5625x the MFMA work. U = G g G^T is formed in double on the host from the
// BN-folded weights; everything on the device is fp32 on v_mfma_f32_16x16x4_f32 (exact fp32 products).
// tools/wino44_precision.py: through the whole network the fp32 F(4x4) logits are within 9e-6 of a
// float64 forward (F(2x2): 8e-6, direct fp32: 7e-6).
//
// Block = 6 waves x one tile group (TR x TC <= 16 tiles, the MFMA M rows) x 48 output channels. Wave i
// owns the Winograd-domain row i (elements (i, 0..5)) and builds its A operands itself: a lane (tile
// t = lane % 16, channel pair k4 = lane / 16) reads the 4 window rows B^T row i touches straight from
// the raw patch (ds_read_b64 = the two input channels of the chunk's two K steps), applies B^T row i,
// then the column transform, and the results ARE its MFMA A registers -- no V tensor through LDS and
// no V barrier (conv_wino_q's limiter). The raw patch of a chunk (8 channels) is
// LDS-DMA'd once per block into a 3-stage ring (one barrier per chunk); U streams from L2 into
// registers one chunk ahead, each register reloaded right after its last MFMA of the chunk (the
// loads then have a whole chunk to land). Epilogue: wave i folds its row with A^T (6 -> 4 values per
// tile and channel), the rows meet in LDS, and Y = A^T (.) with bias and ReLU is stored channels-last
// or 8-channel-blocked (the temporal consumer's layout, engine.hip c8_pair).
#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int W4_WAVES = 6;
constexpr int W4_THREADS = 64 * W4_WAVES;
constexpr int W4_DPW_MAX = 4;                        // LDS-DMA instructions per wave per chunk (3 or 4)
constexpr int W4_STAGE = W4_WAVES * W4_DPW_MAX * 1024;  // 24 KB raw stage (<= 24 x 64 16-B slots used)
constexpr int W4_NR = 3;                                // raw ring stages
constexpr int W4_ZS = 48 * 17 + 1;                   // epilogue plane [co (stride 17)][tile (16)], odd
constexpr int W4_LDS = 24 * W4_ZS * 4;               // 78,432 B: Z[i*4+b] planes; ring + sink inside
static_assert(W4_NR * W4_STAGE + 1024 <= W4_LDS, "ring and sink fit under the epilogue planes");
static_assert(2 * W4_LDS <= 160 * 1024, "two blocks per CU");

__device__ inline int xcd_swizzle4(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// s_waitcnt immediate waiting for vmcnt <= n (gfx9 encoding: vmcnt bits 3:0 and 15:14; expcnt and
// lgkmcnt left at their maxima)
constexpr int vm_wait(int n) { return (n & 0xF) | ((n >> 4) << 14) | 0x0F70; }

}  // namespace

// Tile-group geometry (host-computed, wino4_geometry). Tiles are 4x4 output pixels; a flattened tile
// row is (frame, tile row) = frame * TH + ty, and a group is TR consecutive flattened rows x TC
// consecutive tile columns (segments of different frames are fine: a 1x3x3 conv never mixes frames).
struct W4Geo {
  int TR, TC;   // group shape, TR * TC <= 16 tiles
  int TH, TW;   // tiles per frame column / row
  int RP;       // 16-B LDS slots per raw patch row (a pad slot after every 4 pixels: bank spread)
  int SS;       // slots per segment (>= 6 RP: free slots shift the next segment's banks)
  int RS;       // slots per channel-half region (TR SS); region 1 = input channels 4..7
  int NI;       // DMA wave-instructions carrying data per stage (<= 6 DPW)
  int n_cob;    // 48-channel output blocks
  int gpr;      // groups per flattened tile row (TW / TC)
  FastDiv fd_cob, fd_gpr, fd_th, fd_tc, fd_rp, fd_ss;
};

namespace {

// NCH: input-channel chunks (8 channels each; 0 = runtime). C8: 8-channel-blocked output. DPW: DMA
// instructions per wave per chunk (3: <= 18 per stage; 4: the 8-segment groups of 7x7 maps). KO: timing
// knock-outs for tools/convbench (0 in the product; results are wrong otherwise): 1 no transform
// reads / VALU, 2 no U reloads, 4 no epilogue, 8 no DMAs in the chunk loop; 16 (a variant, correct):
// every window column read from its own address register (no ds_read2_b64 pairing); 32 no chunk barrier.
template <int NCH, bool C8, bool RELU, int DPW, int KO = 0>
__global__ __launch_bounds__(W4_THREADS) __attribute__((amdgpu_waves_per_eu(3, 3))) void conv_wino4(ConvParams p,
                                                                                                     W4Geo g) {
  __shared__ __align__(16) char smem[W4_LDS];
  char* sink = smem + W4_NR * W4_STAGE;

  // buffer descriptors (wave-uniform bases): 32-bit per-lane offsets, no 64-bit address VGPRs; an
  // out-of-range offset reads zeros (the padding pixels)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin * 4), 0x00020000);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int blk = xcd_swizzle4(blockIdx.x, gridDim.x);
  const int grp = fdiv(blk, g.fd_cob), cob = blk - grp * g.n_cob;
  const int rg = fdiv(grp, g.fd_gpr), gx = grp - rg * g.gpr;
  const int R0 = rg * g.TR, tx0 = gx * g.TC;  // first flattened tile row, first tile column
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int nchunk = NCH > 0 ? NCH : C >> 3;
  const int NT = g.TR * g.TC;

  // ---- LDS-DMA slot table: instruction j of this wave fills slots s = (wid + 6 j) * 64 + lane of a
  // stage; s < RS: input channels 0..3 of a pixel, else 4..7; within a region slot = seg * SS + r * RP
  // + cs (window row r < 6 of segment seg), pixel column c = cs - cs / 5 (cs % 5 == 4: pad)
  // (array sized by a constant: a template-dependent bound captured by the lambdas below left the
  // kernels' host stubs undefined under hipcc)
  unsigned d_off[W4_DPW_MAX];  // byte offset of the slot's 16 B in chunk 0, or 0x80000000 (zeros)
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int ins = wid + W4_WAVES * j, s = ins * 64 + lane;
    unsigned off = 0x80000000u;
    if (ins < g.NI && s < 2 * g.RS) {
      const int hf = s >= g.RS ? 1 : 0, sl = s - hf * g.RS;
      const int seg = fdiv(sl, g.fd_ss), ss = sl - seg * g.SS;
      const int r = fdiv(ss, g.fd_rp), cs = ss - r * g.RP;
      const int m5 = cs / 5, k5 = cs - 5 * m5, c = 4 * m5 + k5;
      if (r < 6 && k5 < 4 && c < 4 * g.TC + 2) {
        const int R = R0 + seg, f = fdiv(R, g.fd_th), ty = R - f * g.TH;
        const int yy = 4 * ty - 1 + r, xx = 4 * tx0 - 1 + c;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = (((f * H + yy) * W + xx) * C + hf * 4) * 4;
      }
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int ins = wid + W4_WAVES * j;
      // every wave issues DPW DMAs (wave-uniform vmcnt counts); those past NI land in the sink, the
      // ones past the last chunk re-read chunk 0
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(ins < g.NI ? smem + stage * W4_STAGE + ins * 1024 : sink), 16,
          d_off[j], k < nchunk ? k * 32 : 0, 0, 0);
    }
  };

  // ---- transform lane: tile t (MFMA row), channel pair k4 (MFMA K index) -> region k4 / 2, 8-B half k4 % 2
  const int t = lane & 15, k4 = lane >> 4;
  const int tv = t < NT ? t : 0;  // rows past the group's tiles compute tile 0 again (discarded)
  const int tseg = fdiv(tv, g.fd_tc), tcol = tv - tseg * g.TC;
  const int lane_off = ((k4 >> 1) * g.RS + tseg * g.SS + 5 * tcol) * 16 + (k4 & 1) * 8;
  // B^T row i (Lavin F(4,3)) over window rows (r0..r3) with coefficients (c0..c3): wave-uniform
  int r0, r1, r2, r3;
  float c0, c1, c2, c3;
  switch (wid) {
    case 0: r0 = 0, r1 = 2, r2 = 4, r3 = 4, c0 = 4.f, c1 = -5.f, c2 = 1.f, c3 = 0.f; break;
    case 1: r0 = 1, r1 = 2, r2 = 3, r3 = 4, c0 = -4.f, c1 = -4.f, c2 = 1.f, c3 = 1.f; break;
    case 2: r0 = 1, r1 = 2, r2 = 3, r3 = 4, c0 = 4.f, c1 = -4.f, c2 = -1.f, c3 = 1.f; break;
    case 3: r0 = 1, r1 = 2, r2 = 3, r3 = 4, c0 = -2.f, c1 = -1.f, c2 = 2.f, c3 = 1.f; break;
    case 4: r0 = 1, r1 = 2, r2 = 3, r3 = 4, c0 = 2.f, c1 = -1.f, c2 = -2.f, c3 = 1.f; break;
    default: r0 = 1, r1 = 3, r2 = 5, r3 = 5, c0 = 4.f, c1 = -5.f, c2 = 1.f, c3 = 0.f; break;
  }
  const int ro0 = r0 * g.RP * 16, ro1 = r1 * g.RP * 16, ro2 = r2 * g.RP * 16, ro3 = r3 * g.RP * 16;
  // v[j] = (B^T d B)[i][j] for the lane's tile and its two channels (.x: K step 0, .y: K step 1); the
  // column transform accumulates per window column (each row-pass value dies at once: registers)
  auto transform = [&](int stage, f32x2 (&v)[6]) __attribute__((always_inline)) {
    if constexpr ((KO & 1) != 0) {
#pragma unroll
      for (int j = 0; j < 6; ++j) v[j] = f32x2{(float)(lane + j + stage), (float)(lane - j)};
      return;
    }
    const char* base = smem + stage * W4_STAGE + lane_off;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const int co = (c + (c >> 2)) * 16;  // pixel columns 0..5 of the window -> slots 0,1,2,3,5,6
      const char* b = base + co;
      if constexpr ((KO & 16) != 0) asm volatile("" : "+v"(b));
      const f32x2 d0 = *reinterpret_cast<const f32x2*>(b + ro0);
      const f32x2 d1 = *reinterpret_cast<const f32x2*>(b + ro1);
      const f32x2 d2 = *reinterpret_cast<const f32x2*>(b + ro2);
      const f32x2 d3 = *reinterpret_cast<const f32x2*>(b + ro3);
      const f32x2 t = d0 * c0 + d1 * c1 + d2 * c2 + d3 * c3;
      // B^T columns: c0 (4,0,0,0,0,0) c1 (0,-4,4,-2,2,4) c2 (-5,-4,-4,-1,-1,0) c3 (0,1,-1,2,-2,-5)
      // c4 (1,1,1,1,1,0) c5 (0,0,0,0,0,1)
      switch (c) {
        case 0: v[0] = t * 4.f; break;
        case 1: v[1] = t * -4.f, v[2] = t * 4.f, v[3] = t * -2.f, v[4] = t * 2.f, v[5] = t * 4.f; break;
        case 2: v[0] += t * -5.f, v[1] += t * -4.f, v[2] += t * -4.f, v[3] -= t, v[4] -= t; break;
        case 3: v[1] += t, v[2] -= t, v[3] += t * 2.f, v[4] += t * -2.f, v[5] += t * -5.f; break;
        case 4: v[0] += t, v[1] += t, v[2] += t, v[3] += t, v[4] += t; break;
        default: v[5] += t; break;
      }
    }
  };

  // ---- U operands: [cob][chunk][i][nt][gg][lane][4], component m = 4 gg + comp <-> (j, ks) = (m / 2, m % 2)
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(reinterpret_cast<const float*>(p.w) + ((size_t)cob * nchunk * W4_WAVES + wid) * 2304), (short)0,
      nchunk * W4_WAVES * 2304 * 4, 0x00020000);
  auto load_u = [&](int k, int nt, int gg) __attribute__((always_inline)) {
    return __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(ur, lane * 16, ((k < nchunk ? k : 0) * (W4_WAVES * 2304) + (nt * 3 + gg) * 256) * 4, 0));
  };

  f32x4 acc[6][3];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) acc[j][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 u[3][3];
  f32x2 a[6];

  // ---- prologue: raw(0), raw(1) and U(0) in flight. Per chunk every wave then issues exactly DPW
  // DMAs + 9 U loads (past-the-end ones re-read chunk 0), so the counted vmcnt waits are exact.
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int nt = 0; nt < 3; ++nt)
#pragma unroll
    for (int gg = 0; gg < 3; ++gg) u[nt][gg] = load_u(0, nt, gg);
  __builtin_amdgcn_sched_barrier(0);

  // chunk k (ph = k % 3, compile time: ring stages are immediates): raw(k+2) DMA'd into stage
  // (k+2) % 3 once every wave is past raw(k-1)'s reads; A(k) transformed from stage k % 3 straight
  // into registers; MFMAs on A(k) x U(k), U(k+1) reloaded behind them. Other waves of the SIMD (3 per
  // SIMD, two blocks per CU) fill the matrix pipe while a wave transforms.
  auto step = [&](int k, int ph, bool first) __attribute__((always_inline)) {
    // own raw(k) landed: issued after it are U(k-1), raw(k+1), U(k) (k = 0: raw(1), U(0))
    if (first)
      __builtin_amdgcn_s_waitcnt(vm_wait(DPW + 9));
    else
      __builtin_amdgcn_s_waitcnt(vm_wait(DPW + 18));
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((KO & 32) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((KO & 8) == 0) issue_raw(k + 2, (ph + 2) % W4_NR);
    __builtin_amdgcn_sched_barrier(0);
    transform(ph, a);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int gg = 0; gg < 3; ++gg) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * gg + jj;
            acc[j][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ks ? a[j].y : a[j].x, u[nt][gg][2 * jj + ks], acc[j][nt], 0,
                                                               0, 0);
          }
#pragma unroll
      for (int nt = 0; nt < 3; ++nt)
        if constexpr ((KO & 2) == 0) u[nt][gg] = load_u(k + 1, nt, gg);
    }
    // each group's 3 U reloads right after the 12 MFMAs that read those registers
#pragma unroll
    for (int gg = 0; gg < 3; ++gg) {
      __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);   // VMEM read
    }
  };
  if constexpr (NCH > 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) step(k, k % W4_NR, k == 0);
  } else {
    step(0, 0, true);
    int k = 1;
#pragma unroll 1
    for (; k + 3 <= nchunk; k += 3) {
      step(k, 1, false);
      step(k + 1, 2, false);
      step(k + 2, 0, false);
    }
    if (k < nchunk) step(k, 1, false);
    if (k + 1 < nchunk) step(k + 1, 2, false);
  }
  __builtin_amdgcn_s_waitcnt(vm_wait(0));  // past-the-end DMAs drained before LDS is reused
  __syncthreads();

  if constexpr ((KO & 4) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) sum += acc[j][nt][0] + acc[j][nt][1] + acc[j][nt][2] + acc[j][nt][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  // ---- epilogue: wave i: R_i[b] = sum_j A^T[b][j] M[i][j] -> Z[i*4+b][co][tile]; then
  // Y[a][b] = sum_i A^T[a][i] R_i[b] per unit (tile, 4 channels, column b)
  float* Z = reinterpret_cast<float*>(smem);
  const int q = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int nt = 0; nt < 3; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float m0 = acc[0][nt][r], m1 = acc[1][nt][r], m2 = acc[2][nt][r];
      const float m3 = acc[3][nt][r], m4 = acc[4][nt][r], m5 = acc[5][nt][r];
      const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
      float* zp = Z + (wid * 4) * W4_ZS + (16 * nt + l16) * 17 + 4 * q + r;
      zp[0 * W4_ZS] = m0 + s12 + s34;
      zp[1 * W4_ZS] = d12 + 2.f * d34;
      zp[2 * W4_ZS] = s12 + 4.f * s34;
      zp[3 * W4_ZS] = d12 + 8.f * d34 + m5;
    }
  __syncthreads();
  const int nunits = NT * 48;
  const size_t plane = (size_t)p.N * p.To * H * W * 8;
#pragma unroll
  for (int rnd = 0; rnd < 2; ++rnd) {
    const int un = tid + W4_THREADS * rnd;
    if (un >= nunits) break;
    const int b = un & 3, rest = un >> 2, tile = rest / 12, cq = rest - tile * 12;
    f32x4 z[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const float* zp = Z + (i * 4 + b) * W4_ZS + (4 * cq) * 17 + tile;
      z[i] = f32x4{zp[0], zp[17], zp[34], zp[51]};
    }
    const int seg = fdiv(tile, g.fd_tc), tc = tile - seg * g.TC;
    const int R = R0 + seg, f = fdiv(R, g.fd_th), ty = R - f * g.TH;
    const int xx = 4 * (tx0 + tc) + b, co = cob * 48 + 4 * cq;
    const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s12 = z[1] + z[2], d12 = z[1] - z[2], s34 = z[3] + z[4], d34 = z[3] - z[4];
    f32x4 y[4];
    y[0] = z[0] + s12 + s34;
    y[1] = d12 + 2.f * d34;
    y[2] = s12 + 4.f * s34;
    y[3] = d12 + 8.f * d34 + z[5];
    float* yout = reinterpret_cast<float*>(p.y);
    if (xx >= W) continue;  // partial tiles at the right / bottom edge of maps with H, W % 4 != 0
#pragma unroll
    for (int aa = 0; aa < 4; ++aa) {
      if (4 * ty + aa >= H) break;
      f32x4 o = y[aa] + bias;
      if constexpr (RELU) {
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
      }
      const size_t pix = (size_t)(f * H + 4 * ty + aa) * W + xx;
      const size_t off = C8 ? (size_t)(co >> 3) * plane + pix * 8 + (co & 7) : pix * CO + co;
      *reinterpret_cast<f32x4*>(yout + off) = o;
    }
  }
}

template <int NCH, int DPW>
hipError_t launch_w4(const ConvParams& p, const W4Geo& g, int n_blocks, hipStream_t s) {
  const dim3 grid(n_blocks), block(W4_THREADS);
  if (p.y_c8) {
    if (p.relu)
      hipLaunchKernelGGL((conv_wino4<NCH, true, true, DPW>), grid, block, 0, s, p, g);
    else
      hipLaunchKernelGGL((conv_wino4<NCH, true, false, DPW>), grid, block, 0, s, p, g);
  } else {
    if (p.relu)
      hipLaunchKernelGGL((conv_wino4<NCH, false, true, DPW>), grid, block, 0, s, p, g);
    else
      hipLaunchKernelGGL((conv_wino4<NCH, false, false, DPW>), grid, block, 0, s, p, g);
  }
  return hipGetLastError();
}

// Tile-group shape, patch pitches and DMA count for p (false: no group of >= 12 tiles fits). Tiles
// past the map's right / bottom edge (H, W % 4 != 0) are computed on zero padding and not stored.
bool wino4_geometry(const ConvParams& p, W4Geo* g, int* n_blocks) {
  if (p.Cout % 48 || p.Cin % 8) return false;
  const int TH = (p.Ho + 3) / 4, TW = (p.Wo + 3) / 4;
  const long rows = (long)p.N * p.To * TH;  // flattened tile rows
  int TC = 0;
  for (int d = TW < 16 ? TW : 16; d >= 1 && !TC; --d)
    if (TW % d == 0) TC = d;
  int TR = 0;
  for (int d = 16 / TC; d >= 1 && !TR; --d)
    if (rows % d == 0) TR = d;
  if (TR * TC < 12) return false;
  const int PC = 4 * TC + 2, rp0 = (PC - 1) + (PC - 1) / 4 + 1;
  // RP, SS: fewest tiles sharing a 16-B bank quad of a 256-B row (ds_read_b64: a 32-lane group = 16
  // tiles x one channel pair), then the fewest DMA instructions
  int best = 1 << 30;
  for (int rp = rp0; rp < rp0 + 16; ++rp)
    for (int ss = 6 * rp; ss < 6 * rp + 16; ++ss) {
      const int ni = (2 * TR * ss + 63) / 64;
      if (ni > W4_WAVES * W4_DPW_MAX) continue;
      int cnt[16] = {0}, m = 0;
      for (int t = 0; t < TR * TC; ++t) {
        const int v = ((t / TC) * ss + 5 * (t % TC)) & 15;
        if (++cnt[v] > m) m = cnt[v];
      }
      const int score = m * 1000 + ni;
      if (score < best) best = score, g->RP = rp, g->SS = ss;
    }
  if (best == 1 << 30) return false;
  g->TR = TR, g->TC = TC, g->TH = TH, g->TW = TW;
  g->RS = TR * g->SS;
  g->NI = (2 * g->RS + 63) / 64;
  g->n_cob = p.Cout / 48;
  g->gpr = TW / TC;
  g->fd_cob = fast_div(g->n_cob);
  g->fd_gpr = fast_div(g->gpr);
  g->fd_th = fast_div(TH);
  g->fd_tc = fast_div(TC);
  g->fd_rp = fast_div(g->RP);
  g->fd_ss = fast_div(g->SS);
  *n_blocks = (int)(rows / TR) * g->gpr * g->n_cob;
  return true;
}

}  // namespace

bool wino4_supported(const ConvParams& p) {
  W4Geo g;
  int nb;
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && !p.res && p.KT == 1 && p.KH == 3 && p.KW == 3 &&
         p.sh == 1 && p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Ho == p.Hi &&
         p.Wo == p.Wi && p.To == p.Ti && (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) <
         ((size_t)1 << 31) && wino4_geometry(p, &g, &nb);
}

// p.w: wino4_transform_weights' layout.
hipError_t launch_wino4(const ConvParams& p, hipStream_t s) {
  if (!wino4_supported(p)) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  wino4_geometry(p, &g, &nb);
  switch (p.Cin >> 3) {
    // (launch_w4 called from this non-template function: instantiated from inside another template,
    // hipcc left the kernels' host stubs undefined)
    case 8: return g.NI <= W4_WAVES * 3 ? launch_w4<8, 3>(p, g, nb, s) : launch_w4<8, 4>(p, g, nb, s);
    case 16: return g.NI <= W4_WAVES * 3 ? launch_w4<16, 3>(p, g, nb, s) : launch_w4<16, 4>(p, g, nb, s);
    default: return g.NI <= W4_WAVES * 3 ? launch_w4<0, 3>(p, g, nb, s) : launch_w4<0, 4>(p, g, nb, s);
  }
}

// Every block issues 16 MFMA rows (tiles, the group's padding included) x 36 elements x Cin x 48.
double wino4_exec_gflop(const ConvParams& p) {
  W4Geo g;
  int nb;
  return wino4_geometry(p, &g, &nb) ? 2.0 * nb * 16.0 * 36.0 * p.Cin * 48.0 * 1e-9 : 0.0;
}

// U[cout_p/48][cin_p/8][6 i][3 nt][3 gg][64 lane][4 comp] from folded weights w[cout][cin][3][3] (double):
// lane = k4 * 16 + n, m = 4 gg + comp = 2 j + ks; element (i, j) of G g G^T for input channel
// chunk * 8 + 2 k4 + ks and output channel cob * 48 + nt * 16 + n.
void wino4_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  const int nch = cin_p / 8;
  for (size_t i = 0; i < (size_t)36 * cin_p * cout_p; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* gw = w + ((size_t)o * cin + c) * 9;
      double tmp[6][3];
      for (int i = 0; i < 6; ++i)
        for (int v = 0; v < 3; ++v) tmp[i][v] = G[i][0] * gw[0 * 3 + v] + G[i][1] * gw[1 * 3 + v] + G[i][2] * gw[2 * 3 + v];
      const int cob = o / 48, nt = (o % 48) / 16, n = o % 16;
      const int chunk = c / 8, k4 = (c % 8) / 2, ks = c % 2;
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          const double u = tmp[i][0] * G[j][0] + tmp[i][1] * G[j][1] + tmp[i][2] * G[j][2];
          const int m = 2 * j + ks, gg = m / 4, comp = m % 4;
          U[(((((((size_t)cob * nch + chunk) * 6 + i) * 3 + nt) * 3 + gg) * 64) + k4 * 16 + n) * 4 + comp] = (float)u;
        }
    }
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench: conv_wino4 timing knock-outs (KO bits above) on 8-chunk maps (layer1), channels-last
// output with ReLU.
template <int KO>
static hipError_t launch_w4ko(const ConvParams& p, const W4Geo& g, int nb, hipStream_t s) {
  if (p.Cin == 128)
    hipLaunchKernelGGL((conv_wino4<16, false, true, 3, KO>), dim3(nb), dim3(W4_THREADS), 0, s, p, g);
  else
    hipLaunchKernelGGL((conv_wino4<8, false, true, 3, KO>), dim3(nb), dim3(W4_THREADS), 0, s, p, g);
  return hipGetLastError();
}
hipError_t launch_wino4_ko(const ConvParams& p, hipStream_t s, int ko) {
  W4Geo g;
  int nb;
  if (!wino4_supported(p) || (p.Cin != 64 && p.Cin != 128) || p.y_c8 || !p.relu || !wino4_geometry(p, &g, &nb) || g.NI > 18)
    return hipErrorInvalidValue;
  switch (ko) {
    case 0: return launch_w4ko<0>(p, g, nb, s);
    case 1: return launch_w4ko<1>(p, g, nb, s);
    case 2: return launch_w4ko<2>(p, g, nb, s);
    case 3: return launch_w4ko<3>(p, g, nb, s);
    case 4: return launch_w4ko<4>(p, g, nb, s);
    case 8: return launch_w4ko<8>(p, g, nb, s);
    case 15: return launch_w4ko<15>(p, g, nb, s);
    case 16: return launch_w4ko<16>(p, g, nb, s);
    case 32: return launch_w4ko<32>(p, g, nb, s);
    case 47: return launch_w4ko<47>(p, g, nb, s);
    default: return hipErrorInvalidValue;
  }
}
#endif
