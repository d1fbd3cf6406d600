// Patch-tiled fused Winograd F(2x2, 3x3) for the widest stride-1 1x3x3 fp32 convs (R(2+1)D-18 layer1
// at 32x112x112 clips: 56x56 feature maps; also layer2 of 224x224 clips). Same op, arithmetic and U
// layout as conv_wino (winograd.hip) -- M_e = sum_ci V_e U_e on exact-fp32 v_mfma_f32_16x16x4_f32,
// Y = A^T M A -- with two changes that matter on MI355X:
//  * the 4x4 input windows of a block's tiles are fetched as whole 10x10-pixel patches (a patch =
//    4x4 tiles = 8x8 output pixels): 400 16-B LDS-DMA slots per 8-channel chunk for 32 tiles
//    instead of 32 x 16 pixels = 1024 (2.56x fewer raw bytes through L2 and the TA);
//  * the transform of chunk k+1 is split around the MFMAs of chunk k: its LDS reads are issued
//    before them and its arithmetic and V stores are placed in the MFMA issue gaps
//    (sched_group_barrier), so the matrix pipe no longer idles while a wave transforms.
// Layer1 (30 clips, 64->144): 2.89 -> 2.61 ms (tools/convbench.sh). Maps with Ho, Wo % 8 == 0 use
// 8x8-pixel patches (PT = 4 tiles per side); maps with Ho, Wo % 4 == 0 (layer2 at 112x112 clips:
// 28x28) use 4x4-pixel patches (PT = 2: 8 patches of 6x6 input pixels per block, 1.78x fewer raw
// bytes than per-tile windows; layer2 128->288: conv_wino 1.32 -> 1.18 ms).
#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));


__device__ inline int xcd_swizzle_p(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ inline void dma16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// conv_wino_q: block = 4 waves (wave = transform row i) x 2 patches (32 tiles) x 48 output channels,
// 2 blocks per CU (72 KB LDS); U operands in registers, fetched two chunks ahead (3-way rotation);
// raw ring 3 x 8 KB, V ring 3 x 16 KB so that each chunk's V operands are read into registers one
// chunk ahead (2-way rotation) and the MFMAs start right after the chunk barrier (2.51 -> 2.43 ms on
// layer1). One barrier per chunk.
// Timing probes (round 1): U operands replaced by lane-varying register values cost the same as the
// loads, and loading chunk 0's U every chunk (L1-resident) is no faster: the U fetch is not a
// bottleneck; the MFMA issue stream itself is (SQ_VALU_MFMA_BUSY 57 %).
constexpr int Q_BT = 32;
constexpr int Q_V = 16 * Q_BT * 32;   // 16 KB

// Patch geometry for PT tiles per patch side: PT = 4 (8x8-pixel outputs, 10x10 input; H, W % 8 == 0)
// or PT = 2 (4x4 outputs, 6x6 input: 28x28 maps). A block always holds 32 tiles.
template <int PT>
struct QPatch {
  static constexpr int SIDE = 2 * PT + 2;                 // input patch side (pixels)
  static constexpr int PIX = SIDE * SIDE;
  // pixels between the patches of a raw stage: odd (one pad pixel), so that two patches' pixels of
  // one transform read fall on different 32-B bank quads (see tt below).
  static constexpr int PSTRIDE = PIX + 1;
  static constexpr int PPB = Q_BT / (PT * PT);            // patches per block
  static constexpr int SLOTS = PPB * PSTRIDE * 2;         // 16-B DMA slots per chunk (8 channels)
  static constexpr int DPW = ((SLOTS + 63) / 64 + 3) / 4;  // DMAs per wave per chunk
  // raw stage = all 4*DPW wave-instructions when that still fits 2 blocks per CU, otherwise only the
  // ones carrying data, the rest landing in a 1 KB sink
  static constexpr bool FULL = 3 * (4 * DPW * 1024) + 3 * Q_V <= 80 * 1024;
  static constexpr int NINSTR = FULL ? 4 * DPW : (SLOTS + 63) / 64;
  static constexpr int RAW = NINSTR * 1024;               // raw stage bytes
  static constexpr int LDS = 3 * RAW + 3 * Q_V + (FULL ? 0 : 1024);
};
static_assert(QPatch<4>::LDS == 72 * 1024 && QPatch<4>::DPW == 2, "PT = 4 layout");
static_assert(QPatch<2>::DPW == 3 && QPatch<2>::LDS <= 80 * 1024, "PT = 2 layout: 2 blocks per CU");

// EPI: epilogue form, bit 0 = residual add, bit 1 = ReLU (compile-time: as runtime flags every
// output element carried two selects).
template <int NCH, int PT = 4, int EPI = 2, bool C8 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wino_q(ConvParams p, int n_co,
                                                                                             int n_patches, FastDiv fd_co,
                                                                                             FastDiv fd_frame, FastDiv fd_px) {
  using G = QPatch<PT>;
  constexpr int Q_RAW = G::RAW, DPW = G::DPW;
  __shared__ __align__(16) char smem[G::LDS];
  char* raw = smem;
  char* vbuf = smem + 3 * Q_RAW;
  char* sink = smem + 3 * Q_RAW + 3 * Q_V;  // DMAs past NINSTR (PT = 2) land here

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_p(blockIdx.x, gridDim.x);
  const int bq = fdiv(blk, fd_co);
  const int pg0 = bq * G::PPB, n0 = (blk - bq * n_co) * 48;
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int PY = H / (2 * PT), PX = W / (2 * PT);
  const int nchunk = NCH > 0 ? NCH : C >> 3;

  // raw DMA: instruction j of this wave fills slots s = (wid + 4j)*64 + lane, s = pp*2*PSTRIDE + pix*2 + half
  int d_off[DPW];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int s = (wid + 4 * j) * 64 + lane;
    int off = -1;
    if (s < G::SLOTS) {
      const int pp = s / (2 * G::PSTRIDE), rem = s - pp * (2 * G::PSTRIDE), pix = rem >> 1, half = rem & 1;
      const int py = pix / G::SIDE, px = pix - py * G::SIDE;
      const int gp = pg0 + pp;
      if (gp < n_patches && pix < G::PIX) {
        const int f = fdiv(gp, fd_frame), r = gp - f * (PY * PX);
        const int pr = fdiv(r, fd_px), pc = r - pr * PX;
        const int yy = pr * 2 * PT - 1 + py, xx = pc * 2 * PT - 1 + px;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = ((f * H + yy) * W + xx) * C + half * 4;
      }
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const void* src = (k < nchunk && d_off[j] >= 0) ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      // every wave issues DPW DMAs (wave-uniform vmcnt counts); those past NINSTR go to the sink
      dma16(src, wid + 4 * j < G::NINSTR ? raw + stage * Q_RAW + (wid + 4 * j) * 1024 : sink);
    }
  };
  // U: lane (co = l16, q) of wave (e row) wid, n tile nt: 8 floats U[chunk][wid][co][q][j][s]
  const float* ub = U + (((size_t)wid * CO + n0 + l16) * 4 + q) * 8;
  auto load_u = [&](int k, f32x4 (&u)[3][2]) __attribute__((always_inline)) {
    const float* b = ub + (size_t)(k < nchunk ? k : 0) * 4 * CO * 32;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int h = 0; h < 2; ++h) u[nt][h] = *reinterpret_cast<const f32x4*>(b + (size_t)nt * 16 * 32 + h * 4);
  };
  // transform thread = (tile tt = pp*PT*PT + ly*PT + lx, channel cc)
  // (PT = 2: 8 consecutive tiles per wave; PT = 4: wave = tile row ly of both patches, lane = (lx bit 1, patch, lx bit 0, channel): the
  // ds_read_b32 32-lane groups then hold lx in {0,1} or {2,3} x both patches, whose 32-B slots --
  // 16 lx + 8 pp (mod 32, PSTRIDE = 101) -- cover all 32 banks; lane = (patch, lx, channel) put
  // lx = 0 / 2 and 1 / 3 on the same banks, 2-way)
  // PT = 2: wave = patches 2 wid, 2 wid + 1, lane = (ly, patch bit, lx, channel): a 32-lane group is
  // lx x 2 patches, slots 2 lx + 37 pp (mod 4) all distinct (lane = (patch, ly, lx, channel) put ly = 0
  // and 1 on the same banks)
  const int tt = PT == 4 ? ((lane >> 4) & 1) * 16 + wid * 4 + ((lane >> 3) & 1) + 2 * (lane >> 5)
                         : (2 * wid + ((lane >> 4) & 1)) * 4 + (lane >> 5) * 2 + ((lane >> 3) & 1);
  const int cc = tid & 7;
  const int raw_off = (tt / (PT * PT)) * G::PSTRIDE * 8 + (2 * ((tt / PT) % PT) * G::SIDE + 2 * (tt % PT)) * 8 + cc;
  // V[e][tile&15][(ci>>1) ^ sw][pp][ci&1], sw = ((tile&15) >> 2) & 2: the A-operand ds_read_b128 is
  // serviced in four 16-lane groups ({0-3,12-15,20-27}, ...) that the unswizzled slot order put on 8
  // distinct 16-B bank quads (2-way conflicts); with the swizzle every group covers all 16
  const int v_off = (((tt & 15) * 4 + ((cc >> 1) ^ (((tt & 15) >> 2) & 2))) * 2 + (tt >> 4)) * 2 + (cc & 1);
  auto transform_read = [&](int rstage, float (&d)[16]) __attribute__((always_inline)) {
    const float* rb = reinterpret_cast<const float*>(raw + rstage * Q_RAW) + raw_off;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) d[4 * r + c] = rb[(r * G::SIDE + c) * 8];
  };
  auto transform_write = [&](const float (&d)[16], int vstage) __attribute__((always_inline)) {
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
      t[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
      t[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
      t[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
    float* vb = reinterpret_cast<float*>(vbuf + vstage * Q_V) + v_off;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vb[(4 * r + 0) * Q_BT * 8] = t[4 * r + 0] - t[4 * r + 2];
      vb[(4 * r + 1) * Q_BT * 8] = t[4 * r + 1] + t[4 * r + 2];
      vb[(4 * r + 2) * Q_BT * 8] = t[4 * r + 2] - t[4 * r + 1];
      vb[(4 * r + 3) * Q_BT * 8] = t[4 * r + 1] - t[4 * r + 3];
    }
  };

  f32x4 uu[3][3][2];  // U operands, 3-way rotation (chunk k uses uu[k % 3])
  f32x4 aa[2][4];     // V (A) operands, 2-way rotation (chunk k uses aa[k & 1])
  f32x4 acc[4][2][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) acc[j][m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int a_off = (l16 * 4 + (q ^ ((l16 >> 2) & 2))) * 16;
  auto read_a = [&](int vstage, f32x4 (&a)[4]) __attribute__((always_inline)) {
    const char* vb = vbuf + vstage * Q_V + a_off;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const f32x4*>(vb + (4 * wid + j) * (Q_BT * 32));
  };
  // Pipeline: chunk k multiplies V(k) (operands read into registers during chunk k-1), reads V(k+1),
  // transforms raw(k+2) into V stage (k+2) % 3 and fetches raw(k+4) / U(k+2). The first MFMA after
  // the chunk barrier therefore never waits for LDS.
  // prologue: raw(0..2), U(0); transform raw(0); raw(3) (into raw(0)'s stage, after a barrier), U(1);
  // transform raw(1). Per chunk each wave then issues exactly 2 DMAs + 6 U loads (past-the-end
  // fetches read the zero block / chunk 0), so the counted vmcnt values are exact.
  // (the sched_barriers pin the issue order the counted vmcnt relies on)
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(2, 2);
  __builtin_amdgcn_sched_barrier(0);
  load_u(0, uu[0]);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * DPW + 6));  // raw(0) landed (raw(1), raw(2), U(0) in flight)
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  {
    float d[16];
    transform_read(0, d);
    transform_write(d, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70 | (DPW + 6));  // raw(1) landed (raw(2), U(0) in flight)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();  // every wave has read raw stage 0
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(3, 0);
  __builtin_amdgcn_sched_barrier(0);
  load_u(1, uu[1]);
  __builtin_amdgcn_sched_barrier(0);
  {
    float d[16];
    transform_read(1, d);
    transform_write(d, 1);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own V stores done
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_a(0, aa[0]);

  auto step = [&](int k, f32x4 (&uc)[3][2], f32x4 (&un)[3][2], f32x4 (&ac)[4], f32x4 (&an)[4])
                  __attribute__((always_inline)) {
    // vmcnt(DPW + 6): raw(k+2), U(k) landed; lgkmcnt(0): own V stores and operand reads done
    __builtin_amdgcn_s_waitcnt(0x0070 | (DPW + 6));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // raw(k+4) LDS-DMAs before this chunk's LDS reads: issued after them, the compiler drains the
    // reads (lgkmcnt(0)) in front of the DMA, which stalls the wave's MFMA stream
    issue_raw(k + 4, (k + 1) % 3);
    __builtin_amdgcn_sched_barrier(0);
    read_a((k + 1) % 3, an);
    float d[16];  // raw(k+2) -> V((k+2)%3); branch-free (the last chunks transform unused fetches)
    transform_read((k + 2) % 3, d);
    load_u(k + 2, un);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nt = 0; nt < 3; ++nt) {
            acc[j][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][2 * m + s2], uc[nt][j >> 1][(j & 1) * 2 + s2],
                                                                 acc[j][m][nt], 0, 0, 0);
          }
    transform_write(d, (k + 2) % 3);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // DS read (8 transform, 4 operand)
    }
#pragma unroll
    for (int g = 0; g < DPW + 6; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (DPW LDS-DMAs, 6 U loads)
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  };
  if constexpr (NCH > 0) {
#pragma unroll
    for (int kk = 0; kk < NCH; ++kk) step(kk, uu[kk % 3], uu[(kk + 2) % 3], aa[kk & 1], aa[(kk + 1) & 1]);
  } else {
    int k = 0;
    for (; k + 6 <= nchunk; k += 6) {
#pragma unroll
      for (int i = 0; i < 6; ++i) step(k + i, uu[i % 3], uu[(i + 2) % 3], aa[i & 1], aa[(i + 1) & 1]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (k + i < nchunk) step(k + i, uu[i % 3], uu[(i + 2) % 3], aa[i & 1], aa[(i + 1) & 1]);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain past-the-end fetches before LDS is reused

  // epilogue: unit = (tile, 4 channels); Z[i][tile][co] f32x2 (48 KB) through LDS
  constexpr int CQ = 12, UNITS = Q_BT * CQ, UPT = (UNITS + 255) / 256;
  constexpr bool RES = EPI & 1, RELU = EPI & 2;
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  // output pixel stride: channels-last, or 8-channel blocks [CO/8][pixels][8] (C8 = p.y_c8; a
  // compile-time form: as a runtime flag the PT = 2 instances spilled)
  const int ps = C8 ? 8 : CO;
  const size_t plane = (size_t)n_patches * (4 * PT * PT) * 8;
  size_t u_o[UPT];
  int u_ok[UPT], u_z[UPT];
  f32x4 u_b[UPT], u_r[UPT][4];
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    const int un = tid + 256 * u;
    // channels-last: (tile, 4-channel group) with the groups fastest (192-B runs per pixel); C8:
    // tiles fastest, so a wave's store covers one 8-channel plane's pixels of all 32 tiles and the
    // two 16-B halves of every 32-B pixel come from the same instruction
    const int tl = C8 ? un % Q_BT : un / CQ, cq = C8 ? un / Q_BT : un - tl * CQ;
    const int gp = pg0 + tl / (PT * PT);
    const bool live = un < UNITS && gp < n_patches;
    const int gpc = live ? gp : pg0;
    const int f = fdiv(gpc, fd_frame), r = gpc - f * (PY * PX);
    const int pr = fdiv(r, fd_px), pc = r - pr * PX;
    const int yy = pr * 2 * PT + 2 * ((tl / PT) % PT), xx = pc * 2 * PT + 2 * (tl % PT);
    const int co = n0 + 4 * cq;
    const size_t pix = (size_t)(f * H + yy) * W + xx;
    u_o[u] = C8 ? (co >> 3) * plane + pix * 8 + (co & 7) : pix * CO + co;
    u_z[u] = tl * 48 + 4 * cq;
    u_ok[u] = live;
    u_b[u] = (p.bias && live) ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int px = 0; px < 4; ++px)
      u_r[u][px] = (RES && live) ? *reinterpret_cast<const f32x4*>(res + u_o[u] + (size_t)((px >> 1) * W + (px & 1)) * ps)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x2* zs = reinterpret_cast<f32x2*>(smem);
  __syncthreads();
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float m0 = acc[0][m][nt][r], m1 = acc[1][m][nt][r], m2 = acc[2][m][nt][r], m3 = acc[3][m][nt][r];
        zs[(wid * Q_BT + m * 16 + 4 * q + r) * 48 + nt * 16 + l16] = f32x2{m0 + m1 + m2, m1 - m2 - m3};
      }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    if (!u_ok[u]) continue;
    f32x4 z[4][2];
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const f32x4* zp = reinterpret_cast<const f32x4*>(zs + i2 * Q_BT * 48 + u_z[u]);
      z[i2][0] = zp[0];
      z[i2][1] = zp[1];
    }
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) {
        f32x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int h = c >> 1, e = (c & 1) * 2 + b2;
          const float y = a2 == 0 ? z[0][h][e] + z[1][h][e] + z[2][h][e] : z[1][h][e] - z[2][h][e] - z[3][h][e];
          float o = y + u_b[u][c];
          if constexpr (RES) o += u_r[u][2 * a2 + b2][c];
          if constexpr (RELU) o = relu1(o);
          v[c] = o;
        }
        *reinterpret_cast<f32x4*>(yout + u_o[u] + (size_t)(a2 * W + b2) * ps) = v;
      }
  }
}

template <int NCH, int PT, int EPI>
hipError_t launch_qe(const ConvParams& p, hipStream_t s) {
  constexpr int PPB = QPatch<PT>::PPB;
  const int n_patches = p.N * p.To * (p.Ho / (2 * PT)) * (p.Wo / (2 * PT));
  const int n_co = p.Cout / 48;
  const dim3 grid(((n_patches + PPB - 1) / PPB) * n_co);
  const int px = p.Wo / (2 * PT), py = p.Ho / (2 * PT);
  const FastDiv fd_co = fast_div(n_co), fd_frame = fast_div(px * py), fd_px = fast_div(px);
  if constexpr (EPI == 2) {  // 8-channel-blocked output: the Conv2Plus1D spatial half (engine.hip, c8_pair)
    if (p.y_c8) {
      hipLaunchKernelGGL((conv_wino_q<NCH, PT, EPI, true>), grid, dim3(256), 0, s, p, n_co, n_patches, fd_co, fd_frame,
                         fd_px);
      return hipGetLastError();
    }
  } else {
    if (p.y_c8) return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((conv_wino_q<NCH, PT, EPI, false>), grid, dim3(256), 0, s, p, n_co, n_patches, fd_co, fd_frame,
                     fd_px);
  return hipGetLastError();
}

template <int NCH, int PT = 4>
hipError_t launch_q(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 2: return launch_qe<NCH, PT, 2>(p, s);  // Conv2Plus1D spatial half: BN + ReLU, no residual
    case 3: return launch_qe<NCH, PT, 3>(p, s);
    case 1: return launch_qe<NCH, PT, 1>(p, s);
    default: return launch_qe<NCH, PT, 0>(p, s);
  }
}

}  // namespace

bool winoq_supported(const ConvParams& p) {
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && p.KT == 1 && p.KH == 3 && p.KW == 3 && p.sh == 1 &&
         p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Cin % 8 == 0 && p.Cout % 48 == 0 &&
         p.Ho == p.Hi && p.Wo == p.Wi && p.To == p.Ti && p.Ho % 4 == 0 && p.Wo % 4 == 0 &&
         (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31);
}

// p.w: conv_wino's U layout [Cin/8][4][Cout][4][4][2] (wino_transform_weights).
hipError_t launch_winoq(const ConvParams& p, hipStream_t s) {
  if (!winoq_supported(p)) return hipErrorInvalidValue;
  if (p.Ho % 8 == 0 && p.Wo % 8 == 0) {  // 8x8-pixel patches
    switch (p.Cin >> 3) {
      case 8: return launch_q<8, 4>(p, s);
      case 16: return launch_q<16, 4>(p, s);
      default: return launch_q<0, 4>(p, s);
    }
  }
  switch (p.Cin >> 3) {  // 4x4-pixel patches (28x28 maps)
    case 8: return launch_q<8, 2>(p, s);
    case 16: return launch_q<16, 2>(p, s);
    default: return launch_q<0, 2>(p, s);
  }
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: ko 0 = conv_wino_q, 7 = conv_wino_s (tools/experimental/winograd_s.hip), 8.. = its
// timing variants
hipError_t launch_winos(const ConvParams& p, hipStream_t s);
hipError_t launch_winos_var(const ConvParams& p, hipStream_t s, int var);
hipError_t launch_winoq_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (ko == 7) return launch_winos(p, s);
  if (ko >= 8) return launch_winos_var(p, s, ko - 8);  // ko = 8 + VAR (12: stamps; 20, 28, 36, 44: knock-outs)
  return launch_winoq(p, s);
}
#endif
