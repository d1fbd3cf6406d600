// Barrier-free patch-tiled Winograd F(2x2, 3x3) for the stride-1 1x3x3 fp32 convs on 8x8-pixel
// patches (R(2+1)D-18 layer1 at 32x112x112 clips: 56x56 maps; layer2 at 224x224). Same op, U layout,
// products and accumulation order as conv_wino_q (winograd2.hip) -- the Conv2Plus1D spatial
// conv3d(kernel (1,3,3), padding (0,1,1)) + BN(eval) (+ residual) + ReLU of torchvision's
// r2plus1d_18, called from src/model/R2plus1D_18_MotionNet.py:29-37 -- so the outputs are
// bit-identical to it; what changes is who computes V and who waits for whom.
//
// conv_wino_q shares one transform between its 4 waves: all 256 threads turn the chunk's raw patch
// into V (16 e x 32 tiles x 8 channels) in LDS, and a block barrier per chunk hands it to the waves'
// MFMAs. Measured there: the MFMA pipe idles while the two co-resident blocks' waves of a SIMD sit
// at their chunk barriers. Here wave i (= transform row i, e = 4i..4i+3) computes only the V rows it
// multiplies, straight into its MFMA A operands: row i of B^T d combines two rows of the 4x4 window
// (d0 - d2, d1 + d2, d2 - d1, d1 - d3), so a lane (tile l16 of patch m, channels 2q, 2q+1) reads 2 rows
// x 4 pixels x 8 B per patch (16 ds_read_b64 per chunk) and does 32 VALU ops. Each wave fetches the
// block's whole raw patch pair into its own 2-stage LDS ring (7 LDS-DMA instructions per chunk), so
// no wave ever waits for another until the epilogue's Z exchange: no chunk barriers at all.
//  * stored patch image: pixel (y, x) at y*10 + x + (y >> 1) (one pad pixel after every odd row), its
//    two 16-B halves swapped when (y >> 2) & 1: every ds_read_b64 32-lane group (16 tiles x 2
//    channel pairs) then covers all 64 banks (pixel slot mod 8 = 5 ly + 2 lx + const takes each value
//    for two tile rows ly, ly + 2, whose half-swaps differ);
//  * pipeline per chunk k (NCH compile-time, fully unrolled): vmcnt(7) -> U(k) and raw(k+1) landed
//    (only the previous chunk's 7 raw DMAs may stay in flight); read raw(k+1), the 48 MFMAs of chunk k
//    interleaved with raw(k+1)'s transform into the other A-operand set, U(k+1) into the other U
//    register set (2-way rotation: the 3-way one of conv_wino_q spilled here), then raw(k+3) into the
//    stage just read;
//  * epilogue: conv_wino_q's (Z[i][tile][co] through LDS, one barrier, 16-B stores; 8-channel-blocked
//    output for the temporal kernel when C8).
#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ inline int xcd_swizzle_w4(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

constexpr int W_BT = 32;                   // tiles per block: 2 patches of 4x4 tiles (8x8 output pixels)
constexpr int W_PST = 104;                 // stored pixels per patch (10 x 10 + 4 pads)
constexpr int W_DMA = 7;                   // LDS-DMA instructions per wave and chunk (2 x 104 x 2 = 416 slots)
constexpr int W_STAGE = W_DMA * 1024;      // one wave's raw stage (the 32 surplus slots fetch zeros)
constexpr int W_LDS = 4 * 2 * W_STAGE;     // 4 waves x 2 stages = 56 KiB: two blocks per CU
static_assert(W_LDS >= 4 * W_BT * 48 * 8, "the epilogue's Z exchange reuses the rings");

__device__ __host__ constexpr int wpos(int y, int x) { return y * 10 + x + (y >> 1); }

// s_waitcnt vmcnt(n) (n < 64), lgkmcnt and expcnt unconstrained
template <int N>
__device__ inline void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

template <int NCH, int EPI, bool C8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wino_w(
    ConvParams p, int n_co, int n_patches, FastDiv fd_co, FastDiv fd_frame, FastDiv fd_px) {
  __shared__ __align__(16) char smem[W_LDS];
  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_w4(blockIdx.x, gridDim.x);
  const int bq = fdiv(blk, fd_co);
  const int pg0 = bq * 2, n0 = (blk - bq * n_co) * 48;
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int PY = H >> 3, PX = W >> 3;
  char* ring = smem + wid * 2 * W_STAGE;

  // ---- raw DMA: instruction j, lane -> stored slot s = 64 j + lane = (stored pixel s >> 1, half s & 1)
  int d_off[W_DMA];
#pragma unroll
  for (int j = 0; j < W_DMA; ++j) {
    const int s = 64 * j + lane, sp = s >> 1;
    const int pp = sp >= W_PST ? 1 : 0, pos = sp - pp * W_PST;
    const int rp = pos / 21, rem = pos - 21 * rp;  // row pair: rows 2 rp (10 px), 2 rp + 1 (10 px), pad
    const int y = 2 * rp + (rem >= 10 ? 1 : 0), xpix = rem >= 10 ? rem - 10 : rem;
    const int half = (s & 1) ^ ((y >> 2) & 1);
    const int gp = pg0 + pp;
    int off = -1;
    if (sp < 2 * W_PST && rem < 20 && gp < n_patches) {
      const int f = fdiv(gp, fd_frame), r = gp - f * (PY * PX);
      const int pr = fdiv(r, fd_px), pc = r - pr * PX;
      const int yy = pr * 8 - 1 + y, xx = pc * 8 - 1 + xpix;
      if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = ((f * H + yy) * W + xx) * C + half * 4;
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < W_DMA; ++j) {
      const void* src = (k < NCH && d_off[j] >= 0) ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(ring + stage * W_STAGE + j * 1024),
                                       16, 0, 0);
    }
  };
  // U: lane (co = l16, q) of wave (e row) wid, n tile nt: 8 floats U[chunk][wid][co][q][j][s]
  const float* ub = U + (((size_t)wid * CO + n0 + l16) * 4 + q) * 8;
  auto load_u = [&](int k, f32x4 (&u)[3][2]) __attribute__((always_inline)) {
    const float* b = ub + (size_t)(k < NCH ? k : 0) * 4 * CO * 32;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int h = 0; h < 2; ++h) u[nt][h] = *reinterpret_cast<const f32x4*>(b + (size_t)nt * 16 * 32 + h * 4);
  };

  // ---- this wave's transform row: t = d[ra] + sgn * d[rb] (row i of B^T d), V[i][j] = (t B)[j]
  const int ra = wid == 0 ? 0 : (wid == 2 ? 2 : 1);
  const int rb = wid == 0 ? 2 : (wid == 1 ? 2 : (wid == 2 ? 1 : 3));
  const float sgn = wid == 1 ? 1.f : -1.f;
  // byte address (stage 0) of pixel (2 ly + r, 2 lx) of patch m, channel pair q, for r = ra, rb
  const int ly = l16 >> 2, lx = l16 & 3;
  int rd[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int y = 2 * ly + (h ? rb : ra);
      rd[m][h] = (int)((ring - smem) + ((m * W_PST + wpos(y, 2 * lx)) * 8 + ((((y >> 2) & 1) ^ (q >> 1)) * 4) +
                                        (q & 1) * 2) * 4);
    }
  // raw(k) -> A operands a[j] = {V[4i+j][tile l16][2q], [2q+1], V[..][tile 16 + l16][2q], [2q+1]}
  auto read_raw = [&](int stage, f32x2 (&d)[2][2][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          d[m][h][c] = *reinterpret_cast<const f32x2*>(smem + rd[m][h] + stage * W_STAGE + c * 32);
  };
  auto transform = [&](const f32x2 (&d)[2][2][4], f32x4 (&a)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) t[c] = __builtin_fmaf(sgn, d[m][1][c][s2], d[m][0][c][s2]);  // exact +-
        a[0][2 * m + s2] = t[0] - t[2];
        a[1][2 * m + s2] = t[1] + t[2];
        a[2][2 * m + s2] = t[2] - t[1];
        a[3][2 * m + s2] = t[1] - t[3];
      }
  };

  f32x4 uu[2][3][2];  // U operands, 2-way rotation (chunk k uses uu[k & 1])
  f32x4 aa[2][4];     // A operands, 2-way rotation (chunk k uses aa[k & 1])
  f32x4 acc[4][2][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) acc[j][m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: raw(0) -> stage 0, raw(1) -> stage 1, U(0); V(0); raw(2) -> stage 0.
  // VMEM order from here on: per chunk k, U(k+1) (6) then raw(k+3) (7), so at the top of chunk k only
  // the previous chunk's 7 raw DMAs may still be in flight: U(k) and raw(k+1) have landed.
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  load_u(0, uu[0]);
  __builtin_amdgcn_sched_barrier(0);
  wait_vm<13>();  // raw(0) landed
  __builtin_amdgcn_sched_barrier(0);
  {
    f32x2 d[2][2][4];
    read_raw(0, d);
    transform(d, aa[0]);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): stage 0 read before it is refilled
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(2, 0);
  __builtin_amdgcn_sched_barrier(0);

  auto step = [&](int k, f32x4 (&uc)[3][2], f32x4 (&un)[3][2], f32x4 (&ac)[4], f32x4 (&an)[4])
                  __attribute__((always_inline)) {
    wait_vm<7>();  // U(k), raw(k+1) landed
    __builtin_amdgcn_sched_barrier(0);
    f32x2 d[2][2][4];  // raw(k+1) (past the end: zeros, transformed and never used)
    read_raw((k + 1) & 1, d);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nt = 0; nt < 3; ++nt)
            acc[j][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][2 * m + s2], uc[nt][j >> 1][(j & 1) * 2 + s2],
                                                                 acc[j][m][nt], 0, 0, 0);
    transform(d, an);
    load_u(k + 1, un);
    issue_raw(k + 3, (k + 1) & 1);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read (16 raw)
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU (transform)
    }
#pragma unroll
    for (int g = 0; g < 13; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (6 U loads, 7 LDS-DMAs)
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 11, 0);
  };
#pragma unroll
  for (int kk = 0; kk < NCH; ++kk) step(kk, uu[kk & 1], uu[(kk + 1) & 1], aa[kk & 1], aa[(kk + 1) & 1]);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the past-the-end fetches before LDS is reused

  // ---- epilogue (conv_wino_q's): unit = (tile, 4 channels); Z[i][tile][co] f32x2 (48 KB) through LDS
  constexpr int CQ = 12, UNITS = W_BT * CQ, UPT = (UNITS + 255) / 256;
  constexpr bool RES = EPI & 1, RELU = EPI & 2;
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  const int ps = C8 ? 8 : CO;
  const size_t plane = (size_t)n_patches * 64 * 8;
  size_t u_o[UPT];
  int u_ok[UPT], u_z[UPT];
  f32x4 u_b[UPT], u_r[UPT][4];
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    const int un = tid + 256 * u;
    const int tl = un / CQ, cq = un - tl * CQ;
    const int gp = pg0 + tl / 16;
    const bool live = un < UNITS && gp < n_patches;
    const int gpc = live ? gp : pg0;
    const int f = fdiv(gpc, fd_frame), r = gpc - f * (PY * PX);
    const int pr = fdiv(r, fd_px), pc = r - pr * PX;
    const int yy = pr * 8 + 2 * ((tl / 4) % 4), xx = pc * 8 + 2 * (tl % 4);
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
  __syncthreads();  // every wave is done with its ring
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float m0 = acc[0][m][nt][r], m1 = acc[1][m][nt][r], m2 = acc[2][m][nt][r], m3 = acc[3][m][nt][r];
        zs[(wid * W_BT + m * 16 + 4 * q + r) * 48 + nt * 16 + l16] = f32x2{m0 + m1 + m2, m1 - m2 - m3};
      }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    if (!u_ok[u]) continue;
    f32x4 z[4][2];
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const f32x4* zp = reinterpret_cast<const f32x4*>(zs + i2 * W_BT * 48 + u_z[u]);
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
          if constexpr (RELU) o = fmaxf(o, 0.f);
          v[c] = o;
        }
        *reinterpret_cast<f32x4*>(yout + u_o[u] + (size_t)(a2 * W + b2) * ps) = v;
      }
  }
}

template <int NCH, int EPI>
hipError_t launch_we(const ConvParams& p, hipStream_t s) {
  const int n_patches = p.N * p.To * (p.Ho / 8) * (p.Wo / 8);
  const int n_co = p.Cout / 48;
  const int px = p.Wo / 8, py = p.Ho / 8;
  const FastDiv fd_co = fast_div(n_co), fd_frame = fast_div(px * py), fd_px = fast_div(px);
  const dim3 grid(((n_patches + 1) / 2) * n_co);
  if (p.y_c8)
    hipLaunchKernelGGL((conv_wino_w<NCH, EPI, true>), grid, dim3(256), 0, s, p, n_co, n_patches, fd_co, fd_frame, fd_px);
  else
    hipLaunchKernelGGL((conv_wino_w<NCH, EPI, false>), grid, dim3(256), 0, s, p, n_co, n_patches, fd_co, fd_frame, fd_px);
  return hipGetLastError();
}

template <int NCH>
hipError_t launch_w(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 2: return launch_we<NCH, 2>(p, s);  // Conv2Plus1D spatial half: BN + ReLU, no residual
    case 3: return launch_we<NCH, 3>(p, s);
    case 1: return launch_we<NCH, 1>(p, s);
    default: return launch_we<NCH, 0>(p, s);
  }
}

}  // namespace

// Compile-time chunk counts: Cin = 64 (layer1) and 128 (layer2 at 224x224 clips).
bool winow_supported(const ConvParams& p) {
  return winoq_supported(p) && p.Ho % 8 == 0 && p.Wo % 8 == 0 && (p.Cin == 64 || p.Cin == 128);
}

// p.w: conv_wino's U layout [Cin/8][4][Cout][4][4][2] (wino_transform_weights).
hipError_t launch_winow(const ConvParams& p, hipStream_t s) {
  if (!winow_supported(p)) return hipErrorInvalidValue;
  return p.Cin == 64 ? launch_w<8>(p, s) : launch_w<16>(p, s);
}
