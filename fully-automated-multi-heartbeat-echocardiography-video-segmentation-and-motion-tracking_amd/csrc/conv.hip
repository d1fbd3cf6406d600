// Implicit-GEMM 3-D convolution for the R(2+1)D-18 encoder on gfx950 (fp32 in / fp32 accumulate).
//
// Replaces the cuDNN conv3d + BatchNorm3d(eval) + ReLU (+ residual add) sequences of torchvision's
// r2plus1d_18 (stem, Conv2Plus1D spatial 1x3x3 / temporal 3x1x1, 1x1x1 downsample) called from
// src/model/R2plus1D_18_MotionNet.py:29-37, and the decoder's low-resolution 1x1x1 projections.
//
// Design (MI355X):
//  * activations channels-last [N][T][H][W][C] with C padded to a multiple of 16, so one 16-deep
//    K-slice is 16 contiguous channels of a single tap -> 64-byte coalesced float4 loads; the
//    im2col A tile is gathered on the fly (no materialised im2col);
//  * A (BMx16) and B (BNx16) tiles double-buffered in LDS in a k4-major [4][rows] float4 image:
//    the 16-lane groups of ds_read_b128 then read 16 distinct rows of one 16-B column slot,
//    conflict-free;
//  * v_mfma_f32_16x16x4_f32 (exact fp32, 157 TF chip peak = the VALU peak, but the VALU is left
//    free for the gather address math). Each lane reads one float4 of A and of B per 16-deep slice
//    and issues 4 MFMAs with k permuted (MFMA j of lane group q uses k = 4q + j), so operands are
//    fetched with b128 reads and no shuffles;
//  * epilogue fuses folded-BN bias, residual add and ReLU.
#include "common.h"

namespace {

// XCD-aware tile order: hardware deals blocks round-robin over the 8 XCDs (b % 8 share one L2).
// Give each XCD a contiguous range of logical tiles (bijective for any count), and walk the N tiles
// of one M tile consecutively, so the blocks that re-read an im2col A tile (and the 3x3 halo rows of
// its neighbours) hit the same L2.
__device__ inline int xcd_swizzle(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

template <int MT, int NT, int WM, int WN, int BK, bool SMALLC>
__global__ __launch_bounds__(64 * WM * WN) void conv_igemm_f32(ConvParams p, int n_tiles) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN, NTH = 64 * WM * WN;
  constexpr int KQ = BK / 4;  // float4 columns per tile row
  constexpr int A4 = BM * KQ, B4 = BN * KQ;
  constexpr int AL = (A4 + NTH - 1) / NTH, BL = (B4 + NTH - 1) / NTH;
  __shared__ f32x4 As[2][KQ][BM];
  __shared__ f32x4 Bs[2][KQ][BN];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;

  // Per-thread A-load descriptors (fixed over the K loop).
  int a_n[AL], a_t[AL], a_h[AL], a_w[AL], a_q[AL], a_r[AL];
  bool a_ok[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int e = tid + i * NTH;
    const int r = e / KQ;
    a_r[i] = r;
    a_q[i] = e % KQ;
    int m = m0 + r;
    a_ok[i] = (e < A4) && (m < p.M);
    if (!a_ok[i]) m = 0;
    const int wo = m % p.Wo;
    m /= p.Wo;
    const int ho = m % p.Ho;
    m /= p.Ho;
    const int to = m % p.To;
    a_n[i] = m / p.To;
    a_t[i] = to * p.st - p.pt;
    a_h[i] = ho * p.sh - p.ph;
    a_w[i] = wo * p.sw - p.pw;
  }

  f32x4 ra[AL], rb[BL];
  const int khw = p.KH * p.KW;

  auto load_tiles = [&](int k0) {
    int tap_u = 0, c_u = 0;
    if (!SMALLC) {  // Cin % BK == 0: the whole BK slice lies in one tap
      tap_u = k0 / p.Cin;
      c_u = k0 - tap_u * p.Cin;
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int k = k0 + 4 * a_q[i];
      int tap, c;
      if (SMALLC) {
        tap = k / p.Cin;
        c = k - tap * p.Cin;
      } else {
        tap = tap_u;
        c = c_u + 4 * a_q[i];
      }
      const int kt = tap / khw;
      const int rem = tap - kt * khw;
      const int kh = rem / p.KW;
      const int kw = rem - kh * p.KW;
      const int ti = a_t[i] + kt, hi = a_h[i] + kh, wi = a_w[i] + kw;
      const bool ok = a_ok[i] && (k < p.K) && (unsigned)ti < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi &&
                      (unsigned)wi < (unsigned)p.Wi;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok) {
        const size_t off = ((((size_t)a_n[i] * p.Ti + ti) * p.Hi + hi) * p.Wi + wi) * p.Cin + c;
        v = *reinterpret_cast<const f32x4*>(p.x + off);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * NTH;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < B4) {
        const int r = e / KQ, qq = e % KQ;
        v = *reinterpret_cast<const f32x4*>(p.w + (size_t)(n0 + r) * p.Kp + k0 + 4 * qq);
      }
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i)
      if (tid + i * NTH < A4) As[buf][a_q[i]][a_r[i]] = ra[i];
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * NTH;
      if (e < B4) Bs[buf][e % KQ][e / KQ] = rb[i];
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kp / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tiles((kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      f32x4 a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = As[cur][4 * s + q][wm * 16 * MT + i * 16 + l16];
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = Bs[cur][4 * s + q][wn * 16 * NT + j * 16 + l16];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
    }
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // Epilogue: D[row = 4q + r][col = l16] of each 16x16 tile.
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + wn * 16 * NT + j * 16 + l16;
    if (n >= p.Cout) continue;
    const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 16 * MT + i * 16 + q * 4 + r;
        if (m >= p.M) continue;
        float v = acc[i][j][r] + bv;
        const size_t o = (size_t)m * p.Cout + n;
        if (p.res) v += p.res[o];
        if (p.relu) v = fmaxf(v, 0.f);
        p.y[o] = v;
      }
    }
  }
}

template <int MT, int NT, int WM, int WN, int BK, bool SMALLC>
hipError_t launch_cfg(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_igemm_f32<MT, NT, WM, WN, BK, SMALLC>), dim3(mt * nt), dim3(64 * WM * WN), 0, s, p, nt);
  return hipGetLastError();
}

}  // namespace

int conv_tile_n(int cout_p, int force_nt) {
  const int n16 = cout_p / 16;
  if (force_nt > 0 && n16 % force_nt == 0) return 16 * force_nt;
  for (int nt : {9, 8, 6, 5, 4, 3})
    if (n16 % nt == 0) return 16 * nt;
  return 48;
}

hipError_t launch_conv(const ConvParams& p, int bn, int bk, hipStream_t s) {
  if (p.Cin % 16 != 0) return launch_cfg<2, 3, 4, 1, 16, true>(p, s);
  if (bk == 16) {
    switch (bn) {
      case 48: return launch_cfg<2, 3, 4, 1, 16, false>(p, s);
      case 64: return launch_cfg<2, 4, 4, 1, 16, false>(p, s);
      case 80: return launch_cfg<2, 5, 4, 1, 16, false>(p, s);
      case 96: return launch_cfg<2, 6, 4, 1, 16, false>(p, s);
      case 128: return launch_cfg<2, 8, 4, 1, 16, false>(p, s);
      case 144: return launch_cfg<2, 9, 4, 1, 16, false>(p, s);
    }
  } else {
    switch (bn) {
      case 48: return launch_cfg<2, 3, 4, 1, 32, false>(p, s);
      case 64: return launch_cfg<2, 4, 4, 1, 32, false>(p, s);
      case 80: return launch_cfg<2, 5, 4, 1, 32, false>(p, s);
      case 96: return launch_cfg<2, 6, 4, 1, 32, false>(p, s);
      case 128: return launch_cfg<2, 8, 4, 1, 32, false>(p, s);
      case 144: return launch_cfg<2, 9, 4, 1, 32, false>(p, s);
    }
  }
  return hipErrorInvalidValue;
}

// (N,3,T,H,W) fp32 -> channels-last (N,T,H,W,4) with channel 3 = 0.
__global__ void pack_input_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int T, int HW) {
  const size_t per = (size_t)T * HW;
  const size_t total = (size_t)N * per;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t n = i / per, r = i - n * per;
    const float* src = x + n * 3 * per + r;
    f32x4 v = {src[0], src[per], src[2 * per], 0.f};
    reinterpret_cast<f32x4*>(y)[i] = v;
  }
}

hipError_t launch_pack_input(const float* x, float* y, int N, int T, int HW, hipStream_t s) {
  const size_t total = (size_t)N * T * HW;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_input_kernel, dim3(blocks), dim3(256), 0, s, x, y, N, T, HW);
  return hipGetLastError();
}
