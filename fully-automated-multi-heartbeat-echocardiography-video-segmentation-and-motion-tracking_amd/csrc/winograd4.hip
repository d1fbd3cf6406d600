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
// Block = 4 waves x one tile group (TR x TC <= 16 tiles, the MFMA M rows) x 48 output channels, two
// blocks per CU (one wave of each per SIMD: 6-wave blocks land 2,2,1,1 on the SIMDs and cap even a
// pure MFMA stream at 0.67-0.73 of peak, tools/occ_probe.hip; 4-wave blocks reach 0.93). Wave
// (rh, ch) owns the 3 x 3 quadrant of Winograd-domain elements (3 rh + r, 3 ch + jj) and builds its
// own A operands: a lane (tile t = lane % 16, channel pair k4 = lane / 16) reads the 5 window rows
// its B^T rows touch straight from the raw patch (ds_read_b64 = the two input channels of the
// chunk's two K steps), applies its 3 B^T rows, then its 3 columns of the column transform; the
// results ARE its MFMA A registers -- no V tensor through LDS and no V barrier (conv_wino_q's
// limiter). The raw patch of a chunk (8 channels) is LDS-DMA'd once per block
// into a ring (one barrier per chunk, or per 2 chunks with a 4-stage ring); U streams from L2 into
// registers one chunk ahead, each register reloaded right after the MFMAs that read it (the loads
// then have a whole chunk to land). On gfx950 the f32 VALU and the f32 MFMA share one rate, so the
// transforms' packed-f32 work is priced in MFMA cycles (about 15 % of them). Epilogue, per 16
// output channels: each wave folds its 3 columns with A^T (the distinct partial sums only), the
// halves meet in LDS, and Y = A^T (.) A with bias and ReLU is stored channels-last or
// 8-channel-blocked (the temporal consumer's layout, engine.hip c8_pair).
#include <type_traits>

#include "wino4_common.h"

namespace {

// NCH: input-channel chunks (8 channels each; 0 = runtime). C8: 8-channel-blocked output. DPW: DMA
// instructions per wave per chunk (W4Ring). KO: timing knock-outs for tools/convbench (0 in the product;
// results are wrong otherwise): 1 no transform reads / VALU, 2 no U reloads, 4 no epilogue, 8 no DMAs
// in the chunk loop, 16 no transform reads (its VALU kept), 32 no chunk barrier; 64 n: the first round's second blocks sleep n x 8128 cycles.
template <int NCH, bool C8, bool RELU, int DPW, int KO = 0>
__global__ __launch_bounds__(W4_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wino4(ConvParams p,
                                                                                                     W4Geo g) {
  using RG = W4Ring<DPW>;
  constexpr int NR = RG::NR, STAGE = RG::STAGE;
  __shared__ __align__(16) char smem[RG::LDS];
  char* sink = smem + NR * STAGE;

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

  // ---- LDS-DMA slot table: instruction j of this wave fills slots s = (wid + 4 j) * 64 + lane of a
  // stage; s < RS: input channels 0..3 of a pixel, else 4..7; within a region slot = seg * SS + r * RP
  // + cs (window row r < 6 of segment seg), pixel column c = cs - cs / 5 (cs % 5 == 4: pad)
  unsigned d_off[6];  // byte offset of the slot's 16 B in chunk 0, or 0x80000000 (zeros)
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
          xr, (__attribute__((address_space(3))) void*)(ins < g.NI ? smem + stage * STAGE + ins * 1024 : sink), 16,
          d_off[j], k < nchunk ? k * 32 : 0, 0, 0);
    }
  };

  // ---- transform lane: tile t (MFMA row), channel pair k4 (MFMA K index) -> region k4 / 2, 8-B half k4 % 2
  const int rh = wid >> 1, ch = wid & 1;
  const int t = lane & 15, k4 = lane >> 4;
  const int tv = t < NT ? t : 0;  // rows past the group's tiles compute tile 0 again (discarded)
  const int tseg = fdiv(tv, g.fd_tc), tcol = tv - tseg * g.TC;
  const int lane_off = ((k4 >> 1) * g.RS + tseg * g.SS + rh * g.RP + 5 * tcol) * 16 + (k4 & 1) * 8;
  const int rp16 = g.RP * 16;
  // a[r][jj] = (B^T d B)[3 rh + r][3 ch + jj] for the lane's tile and its two channels (.x: K step 0,
  // .y: K step 1). One straight-line body per quadrant (a wave-uniform switch per chunk): the 30 reads
  // are scheduled ahead of their arithmetic instead of waiting column by column.
  auto transform = [&](int stage, f32x2 (&a)[3][3]) __attribute__((always_inline)) {
    if constexpr ((KO & 1) != 0) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) a[r][jj] = f32x2{(float)(lane + 3 * r + jj + stage), (float)(lane - jj)};
      return;
    }
    const char* base = smem + stage * STAGE + lane_off;
    auto body = [&](auto rh_c, auto ch_c) __attribute__((always_inline)) {
      constexpr int RH = decltype(rh_c)::value, CH = decltype(ch_c)::value;
      f32x2 tt[3][6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int co = (c + (c >> 2)) * 16;  // pixel columns 0..5 of the window -> slots 0,1,2,3,5,6
        f32x2 e[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          if constexpr ((KO & 16) != 0)  // probe: the transform's VALU without its LDS reads
            e[q] = f32x2{(float)(lane + q + c + stage), (float)(lane * q - c)};
          else
            e[q] = *reinterpret_cast<const f32x2*>(base + q * rp16 + co);
        }
        f32x2 t3[3];
        bt_rows<RH>(e, t3);
#pragma unroll
        for (int r = 0; r < 3; ++r) tt[r][c] = t3[r];
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) bt_cols<CH>(tt[r], a[r]);
    };
    switch (wid) {
      case 0: body(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}); break;
      case 1: body(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}); break;
      case 2: body(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}); break;
      default: body(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}); break;
    }
  };

  // ---- U operands: [cob][chunk][wave][14][lane][4]; component m = 4 g + comp <-> MFMA (r, ks, nt, jj),
  // m = ((r * 2 + ks) * 3 + nt) * 3 + jj (m >= 54: zero pad)
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(reinterpret_cast<const float*>(p.w) + ((size_t)cob * nchunk * W4_WAVES + wid) * (W4_NU * 256)),
      (short)0, nchunk * W4_WAVES * W4_NU * 256 * 4, 0x00020000);
  auto load_u = [&](int k, int gi) __attribute__((always_inline)) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         ur, lane * 16, ((k < nchunk ? k : 0) * (W4_WAVES * W4_NU * 256) + gi * 256) * 4, 0));
  };

  f32x4 acc[3][3][3];  // [r][jj][nt]
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) acc[r][jj][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 u[W4_NU];
  f32x2 a[3][3];

  if constexpr ((KO & 64) != 0) {  // stagger probe: the second block of each CU in the first round starts late
    if (blockIdx.x >= 256 && blockIdx.x < 512)
      for (int i = 0; i < (KO & 4095) / 64; ++i) __builtin_amdgcn_s_sleep(127);
  }
  if constexpr ((KO & 4096) != 0) {  // the same with the odd blocks of the first round
    if ((blockIdx.x & 1) && blockIdx.x < 512)
      for (int i = 0; i < 2; ++i) __builtin_amdgcn_s_sleep(127);
  }
  // ---- prologue: raw(0), raw(1) and U(0) in flight. Per chunk every wave then issues exactly DPW
  // DMAs + 14 U loads (past-the-end ones re-read chunk 0), so the counted vmcnt waits are exact.
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int gi = 0; gi < W4_NU; ++gi) u[gi] = load_u(0, gi);
  __builtin_amdgcn_sched_barrier(0);

  // chunk k (ph = k % NR, compile time: ring stages are immediates). Every STEP chunks (a barrier):
  // raw(k+2) .. raw(k+NR-1) DMA'd into the stages of chunks k-STEP .. k-1, which every wave has read
  // once it is past the barrier. A(k) transformed from stage ph straight into registers; MFMAs on
  // A(k) x U(k), U(k+1) reloaded behind them; the other block's wave on the SIMD fills the matrix
  // pipe while this one transforms.
  auto step = [&](int k, int ph, bool first) __attribute__((always_inline)) {
    if (ph % RG::STEP == 0) {
      // own raw(k) .. raw(k+STEP-1) landed: issued after them are the U loads of the STEP chunks
      // before k (NR = 3 also raw(k+1)); first: U(0) only (NR = 3: raw(1), U(0))
      constexpr int AFTER = NR == 3 ? DPW + W4_NU : W4_NU;
      if (first)
        __builtin_amdgcn_s_waitcnt(vm_wait(AFTER));
      else
        __builtin_amdgcn_s_waitcnt(vm_wait(AFTER + W4_NU));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((KO & 32) == 0) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((KO & 8) == 0) {
#pragma unroll
        for (int d = 2; d < NR; ++d) issue_raw(k + d, (ph + d) % NR);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    transform(ph, a);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 54; ++m) {
      const int jj = m % 3, nt = (m / 3) % 3, ks = (m / 9) % 2, r = m / 18;
      acc[r][jj][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ks ? a[r][jj].y : a[r][jj].x, u[m >> 2][m & 3],
                                                            acc[r][jj][nt], 0, 0, 0);
      if ((m & 3) == 3 || m == 53) {
        if constexpr ((KO & 2) == 0) u[m >> 2] = load_u(k + 1, m >> 2);
      }
    }
    if constexpr ((KO & 2) == 0) u[W4_NU - 1] = load_u(k + 1, W4_NU - 1);  // (the all-pad group: count only)
    // each group's reload right after the 4 MFMAs that read it
#pragma unroll
    for (int gi = 0; gi < W4_NU - 2; ++gi) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
  };
  if constexpr (NCH > 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) step(k, k % NR, k == 0);
  } else {
    // one ring revolution per loop trip (a fully unrolled runtime-length loop is not possible)
#pragma unroll
    for (int k = 0; k < NR - 1; ++k)
      if (k < nchunk) step(k, k, k == 0);
    int k = NR - 1;
#pragma unroll 1
    for (; k + NR <= nchunk; k += NR) {
#pragma unroll
      for (int i = 0; i < NR; ++i) step(k + i, (NR - 1 + i) % NR, false);
    }
#pragma unroll
    for (int i = 0; i < NR - 1; ++i)
      if (k + i < nchunk) step(k + i, (NR - 1 + i) % NR, false);
  }
  __builtin_amdgcn_s_waitcnt(vm_wait(0));  // past-the-end DMAs and U loads drained before LDS is reused

  if constexpr ((KO & 4) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          sum += acc[r][jj][nt][0] + acc[r][jj][nt][1] + acc[r][jj][nt][2] + acc[r][jj][nt][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  // ---- epilogue, per 16 output channels nt: wave (rh, ch) stores the column partial sums of its rows
  // i = 3 rh + r, P[i][b] = sum_j A^T[b][j] M[i][j] = E[e(b)] + F[b]: ch 0 the distinct E = (m0+m1+m2,
  // m1-m2, m1+m2) (e(b) = 0, 1, 2, 1), ch 1 F = (m3+m4, 2(m3-m4), 4(m3+m4), 8(m3-m4)+m5); a thread then
  // owns one unit (tile, 4 channels, column b) and stores Y[a][b] = sum_i A^T[a][i] P[i][b], a = 0..3.
  float* Z = reinterpret_cast<float*>(smem);
  const int q = lane >> 4, l16 = lane & 15;
  const size_t plane = (size_t)p.N * p.To * H * W * 8;
  float* yout = reinterpret_cast<float*>(p.y);
  const int ub = tid & 3, ucq = (tid >> 2) & 3, utile = tid >> 4;  // this thread's unit
  const int useg = fdiv(utile, g.fd_tc), utc = utile - useg * g.TC;
  const int uR = R0 + useg, uf = fdiv(uR, g.fd_th), uty = uR - uf * g.TH;
  const int uxx = 4 * (tx0 + utc) + ub;
  const bool ulive = utile < NT && uxx < W;
  // the 3 N tiles' bias vectors before the first store, one explicit vmcnt(0): a bias load after a
  // store waits for it (vmcnt retires in order), once per N tile in the per-tile form
  f32x4 biasv[3];
#pragma unroll
  for (int nt = 0; nt < 3; ++nt)
    biasv[nt] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + cob * 48 + nt * 16 + 4 * ucq) : f32x4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
  for (int nt = 0; nt < 3; ++nt) {
    __syncthreads();  // the ring (nt = 0) / the previous pass's planes are no longer read
    if (ch == 0) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const f32x4 m0 = acc[r][0][nt], m1 = acc[r][1][nt], m2 = acc[r][2][nt];
        f32x4* zp = reinterpret_cast<f32x4*>(Z + ((3 * rh + r) * 3) * W4_ZS + l16 * W4_CS + 4 * q);
        zp[0] = m0 + m1 + m2;
        zp[W4_ZS / 4] = m1 - m2;
        zp[2 * W4_ZS / 4] = m1 + m2;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const f32x4 m0 = acc[r][0][nt], m1 = acc[r][1][nt], m2 = acc[r][2][nt];
        f32x4* zp = reinterpret_cast<f32x4*>(Z + (18 + (3 * rh + r) * 4) * W4_ZS + l16 * W4_CS + 4 * q);
        const f32x4 sm = m0 + m1, df = m0 - m1;
        zp[0] = sm;
        zp[W4_ZS / 4] = 2.f * df;
        zp[2 * W4_ZS / 4] = 4.f * sm;
        zp[3 * W4_ZS / 4] = 8.f * df + m2;
      }
    }
    __syncthreads();
    if constexpr ((KO & 32768) != 0) {
      // probe (correct results): unit = (channel, column b, 4 tiles) -- 16-B plane reads over 4 tiles
      // instead of 4-B reads over 4 channels, one 4-B store per (tile, row)
      const int c16 = tid & 15, vb = (tid >> 4) & 3, tg = tid >> 6;
      const int veb = vb == 3 ? 1 : vb;
      f32x4 P[6];
#pragma unroll
      for (int i = 0; i < 6; ++i)
        P[i] = *reinterpret_cast<const f32x4*>(Z + (i * 3 + veb) * W4_ZS + c16 * W4_CS + 4 * tg) +
               *reinterpret_cast<const f32x4*>(Z + (18 + i * 4 + vb) * W4_ZS + c16 * W4_CS + 4 * tg);
      const int co = cob * 48 + nt * 16 + c16;
      const float bias = p.bias ? p.bias[co] : 0.f;
      const f32x4 s12 = P[1] + P[2], d12 = P[1] - P[2], s34 = P[3] + P[4], d34 = P[3] - P[4];
      f32x4 y[4];
      y[0] = P[0] + s12 + s34;
      y[1] = d12 + 2.f * d34;
      y[2] = s12 + 4.f * s34;
      y[3] = d12 + 8.f * d34 + P[5];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int tile = 4 * tg + tt;
        const int vseg = fdiv(tile, g.fd_tc), vtc = tile - vseg * g.TC;
        const int vR = R0 + vseg, vf = fdiv(vR, g.fd_th), vty = vR - vf * g.TH;
        const int vxx = 4 * (tx0 + vtc) + vb;
        if (tile >= NT || vxx >= W) continue;
#pragma unroll
        for (int aa = 0; aa < 4; ++aa) {
          if (4 * vty + aa >= H) break;
          float o = y[aa][tt] + bias;
          if constexpr (RELU) o = relu1(o);
          const size_t pix = (size_t)(vf * H + 4 * vty + aa) * W + vxx;
          yout[C8 ? (size_t)(co >> 3) * plane + pix * 8 + (co & 7) : pix * CO + co] = o;
        }
      }
      continue;
    }
    if (ulive) {
      f32x4 P[6];
      const int eb = ub == 3 ? 1 : ub;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float* e = Z + (i * 3 + eb) * W4_ZS + (4 * ucq) * W4_CS + utile;
        const float* f = Z + (18 + i * 4 + ub) * W4_ZS + (4 * ucq) * W4_CS + utile;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if constexpr ((KO & 16384) != 0)  // probe: no unit LDS reads
            P[i][c] = (float)(i + c + utile);
          else
            P[i][c] = e[c * W4_CS] + f[c * W4_CS];
        }
      }
      const int co = cob * 48 + nt * 16 + 4 * ucq;
      const f32x4 bias = biasv[nt];
      const f32x4 s12 = P[1] + P[2], d12 = P[1] - P[2], s34 = P[3] + P[4], d34 = P[3] - P[4];
      f32x4 y[4];
      y[0] = P[0] + s12 + s34;
      y[1] = d12 + 2.f * d34;
      y[2] = s12 + 4.f * s34;
      y[3] = d12 + 8.f * d34 + P[5];
#pragma unroll
      for (int aa = 0; aa < 4; ++aa) {
        if (4 * uty + aa >= H) break;  // partial tiles at the bottom edge (H % 4 != 0)
        f32x4 o = y[aa] + bias;
        if constexpr (RELU) {
#pragma unroll
          for (int c = 0; c < 4; ++c) o[c] = relu1(o[c]);
        }
        const size_t pix = (size_t)(uf * H + 4 * uty + aa) * W + uxx;
        const size_t off = C8 ? (size_t)(co >> 3) * plane + pix * 8 + (co & 7) : pix * CO + co;
        if constexpr ((KO & 8192) != 0) {  // probe: no output stores
          if (o[0] == 1234.5f) *reinterpret_cast<f32x4*>(yout + off) = o;
        } else if constexpr ((KO & 65536) != 0) {  // probe: non-temporal output stores
          __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(yout + off));
        } else {
          *reinterpret_cast<f32x4*>(yout + off) = o;
        }
      }
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

}  // namespace

// tile groups: the most tiles per group (16 fills every MFMA row), then the widest (28x28 maps: 16 x 1
// instead of 2 x 7); wino4_geometry
constexpr int W4_FILL = 1;

bool wino4_supported(const ConvParams& p) {
  W4Geo g;
  int nb;
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && !p.res && p.KT == 1 && p.KH == 3 && p.KW == 3 &&
         p.sh == 1 && p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Ho == p.Hi &&
         p.Wo == p.Wi && p.To == p.Ti && (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) <
         ((size_t)1 << 31) && wino4_geometry(p, &g, &nb, 48, W4_FILL);
}

// p.w: wino4_transform_weights' layout. (The launch templates are called from this non-template
// function: instantiated from inside another template, hipcc left the kernels' host stubs undefined.)
hipError_t launch_wino4(const ConvParams& p, hipStream_t s) {
  if (!wino4_supported(p)) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  wino4_geometry(p, &g, &nb, 48, W4_FILL);
  const int dpw = (g.NI + W4_WAVES - 1) / W4_WAVES;
  switch (p.Cin >> 3) {
    case 8:
      return dpw <= 4 ? launch_w4<8, 4>(p, g, nb, s) : dpw == 5 ? launch_w4<8, 5>(p, g, nb, s) : launch_w4<8, 6>(p, g, nb, s);
    case 16:
      return dpw <= 4 ? launch_w4<16, 4>(p, g, nb, s)
                      : dpw == 5 ? launch_w4<16, 5>(p, g, nb, s) : launch_w4<16, 6>(p, g, nb, s);
    default:
      return dpw <= 4 ? launch_w4<0, 4>(p, g, nb, s) : dpw == 5 ? launch_w4<0, 5>(p, g, nb, s) : launch_w4<0, 6>(p, g, nb, s);
  }
}

// Every block issues 16 MFMA rows (tiles, the group's padding included) x 36 elements x Cin x 48.
double wino4_exec_gflop(const ConvParams& p) {
  W4Geo g;
  int nb;
  return wino4_geometry(p, &g, &nb, 48, W4_FILL) ? 2.0 * nb * 16.0 * 36.0 * p.Cin * 48.0 * 1e-9 : 0.0;
}

// U[cout_p/48][cin_p/8][4 waves][14][64 lane][4] from folded weights w[cout][cin][3][3] (double): wave
// w = (rh, ch) = (w / 2, w % 2), lane = k4 * 16 + n, component m = 4 g + comp = ((r * 2 + ks) * 3 + nt)
// * 3 + jj (m >= 54: zero); element (3 rh + r, 3 ch + jj) of G g G^T for input channel chunk * 8 +
// 2 k4 + ks and output channel cob * 48 + nt * 16 + n.
void wino4_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  const int nch = cin_p / 8, ncob = cout_p / 48;
  const size_t total = (size_t)ncob * nch * W4_WAVES * W4_NU * 256;
  for (size_t i = 0; i < total; ++i) U[i] = 0.f;
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
          const int wv = (i / 3) * 2 + j / 3, r = i % 3, jj = j % 3;
          const int m = ((r * 2 + ks) * 3 + nt) * 3 + jj, gi = m / 4, comp = m % 4;
          U[((((((size_t)cob * nch + chunk) * W4_WAVES + wv) * W4_NU + gi) * 64) + k4 * 16 + n) * 4 + comp] = (float)u;
        }
    }
}

// Floats of wino4_transform_weights' output for a cin_p x cout_p conv.
size_t wino4_weight_floats(int cin_p, int cout_p) {
  return (size_t)(cout_p / 48) * (cin_p / 8) * W4_WAVES * W4_NU * 256;
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench: conv_wino4 timing knock-outs (KO bits above) on 8- or 16-chunk maps, channels-last
// output with ReLU.
template <int KO>
static hipError_t launch_w4ko(const ConvParams& p, const W4Geo& g, int nb, hipStream_t s) {
  if (p.Cin == 128)
    hipLaunchKernelGGL((conv_wino4<16, false, true, 4, KO>), dim3(nb), dim3(W4_THREADS), 0, s, p, g);
  else
    hipLaunchKernelGGL((conv_wino4<8, false, true, 4, KO>), dim3(nb), dim3(W4_THREADS), 0, s, p, g);
  return hipGetLastError();
}
hipError_t launch_wino4_ko(const ConvParams& p, hipStream_t s, int ko) {
  W4Geo g;
  int nb;
  if (!wino4_supported(p) || (p.Cin != 64 && p.Cin != 128) || p.y_c8 || !p.relu || !wino4_geometry(p, &g, &nb, 48, W4_FILL) ||
      g.NI > 16)
    return hipErrorInvalidValue;
  switch (ko) {
    case 1: return launch_w4ko<1>(p, g, nb, s);
    case 2: return launch_w4ko<2>(p, g, nb, s);
    case 3: return launch_w4ko<3>(p, g, nb, s);
    case 4: return launch_w4ko<4>(p, g, nb, s);
    case 8: return launch_w4ko<8>(p, g, nb, s);
    case 15: return launch_w4ko<15>(p, g, nb, s);
    case 32: return launch_w4ko<32>(p, g, nb, s);
    case 47: return launch_w4ko<47>(p, g, nb, s);
    case 16: return launch_w4ko<16>(p, g, nb, s);
    case 64: return launch_w4ko<64>(p, g, nb, s);
    case 128: return launch_w4ko<128>(p, g, nb, s);
    case 192: return launch_w4ko<192>(p, g, nb, s);
    case 256: return launch_w4ko<256>(p, g, nb, s);
    case 4096: return launch_w4ko<4096>(p, g, nb, s);
    case 8192: return launch_w4ko<8192>(p, g, nb, s);
    case 16384: return launch_w4ko<16384>(p, g, nb, s);
    case 24576: return launch_w4ko<24576>(p, g, nb, s);
    case 32768: return launch_w4ko<32768>(p, g, nb, s);
    case 65536: return launch_w4ko<65536>(p, g, nb, s);
    default: return launch_w4ko<0>(p, g, nb, s);
  }
}
#endif
