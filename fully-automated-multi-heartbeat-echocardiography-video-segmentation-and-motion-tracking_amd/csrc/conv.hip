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

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant (Cin % 16 == 0): the A (im2col gather) and B tiles of each 16-deep K step are
// copied global -> LDS by global_load_lds_dwordx4 (no VGPR staging) into an S-stage ring, so S-1
// K steps of loads are in flight while the MFMAs of the current one run. Waits are counted per
// wave (s_waitcnt vmcnt(N) with N = loads issued after the stage being consumed) followed by a raw
// s_barrier; __syncthreads() would drain every DMA (vmcnt(0)).
// Tile image per stage: rows of 64 B (16 floats of K), row-major, A rows then B rows; the 16-B
// slot of (row, q) is stored at q ^ g[(row >> 2) & 3] with g = {0, 2, 3, 1}: every ds_read_b128
// lane group then touches 16 distinct bank quads (checked exhaustively). DMA writes are lane
// linear, so the swizzle is applied to the per-lane SOURCE address (the inverse permutation).
// Padding taps (conv borders) and rows past M read a 16-B zero block instead.
template <int MT, int NT, int S>
__global__ __launch_bounds__(256) void conv_dma_f32(ConvParams p, int n_tiles) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  constexpr int A_INS = BM / 16, B_INS = BN / 16, T_INS = A_INS + B_INS;
  constexpr int PER_WAVE = (T_INS + 3) / 4;
  constexpr int STAGE = T_INS * 1024;           // bytes per ring stage
  constexpr int JUNK = S * STAGE;               // 1 KB sink for the padding DMAs
  __shared__ __align__(16) char smem[S * STAGE + 1024];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;
  constexpr int G[4] = {0, 2, 3, 1};

  // ---- per-lane DMA descriptors: lane writes row (lane >> 2), physical slot (lane & 3)
  const int drow = lane >> 2;
  const int dq = (lane & 3) ^ G[(drow >> 2) & 3];  // logical 16-B slot this lane fetches
  const float* d_base[PER_WAVE];
  int d_t[PER_WAVE], d_h[PER_WAVE], d_w[PER_WAVE], d_pix[PER_WAVE], d_kind[PER_WAVE];  // kind 0 A, 1 B, 2 junk
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int idx = wid + 4 * j;
    d_t[j] = d_h[j] = d_w[j] = d_pix[j] = 0;
    d_base[j] = p.zero;
    if (idx < A_INS) {
      d_kind[j] = 0;
      int m = m0 + idx * 16 + drow;
      const bool ok = m < p.M;
      if (!ok) m = 0;
      const int wo = m % p.Wo;
      m /= p.Wo;
      const int ho = m % p.Ho;
      m /= p.Ho;
      const int to = m % p.To;
      d_t[j] = ok ? to * p.st - p.pt : -(1 << 20);  // a row past M never passes the bounds test
      d_h[j] = ho * p.sh - p.ph;
      d_w[j] = wo * p.sw - p.pw;
      // linear input-voxel index of tap (0,0,0); may point outside when padded (never used then)
      d_pix[j] = (((m / p.To) * p.Ti + d_t[j]) * p.Hi + d_h[j]) * p.Wi + d_w[j];
    } else if (idx < T_INS) {
      d_kind[j] = 1;
      d_base[j] = p.w + (size_t)(n0 + (idx - A_INS) * 16 + drow) * p.Kp + 4 * dq;
    } else {
      d_kind[j] = 2;
    }
  }
  const int khw = p.KH * p.KW;
  const int kmain = p.KT * khw * p.Cin;  // K columns from x; the rest (1x1 dual input) from x2

  auto issue = [&](int k_step, int slot) {
    const int k0 = k_step * 16;
    const bool second = k0 >= kmain;
    const int cin = second ? p.Cin2 : p.Cin;
    const float* xb = second ? p.x2 : p.x;
    const int kk0 = second ? k0 - kmain : k0;
    const int tap = kk0 / cin, c0 = kk0 - tap * cin;
    const int kt = tap / khw, rem = tap - kt * khw, kh = rem / p.KW, kw = rem - kh * p.KW;
    const int tap_pix = (kt * p.Hi + kh) * p.Wi + kw;
    const float* xc = xb + c0 + 4 * dq;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int idx = wid + 4 * j;
      const float* src;
      if (d_kind[j] == 0) {
        const int ti = d_t[j] + kt, hi = d_h[j] + kh, wi = d_w[j] + kw;
        const bool ok = (unsigned)ti < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi;
        src = ok ? xc + (size_t)(unsigned)(d_pix[j] + tap_pix) * cin : p.zero;
      } else if (d_kind[j] == 1) {
        src = d_base[j] + k0;
      } else {
        src = p.zero;
      }
      char* dst = (idx < T_INS) ? smem + slot * STAGE + idx * 1024 : smem + JUNK;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kp / 16;
  // prologue: stages 0 .. S-2
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);

  const int pq = q ^ G[l16 >> 2];  // physical slot of this lane's fragment reads
  const int a_off = (wid * 16 * MT + l16) * 64 + pq * 16;
  const int b_off = A_INS * 1024 + l16 * 64 + pq * 16;
  for (int k = 0; k < nk; ++k) {
    // stage k landed (this wave's DMAs), then every wave's (barrier); also: everyone is done
    // reading stage k-1, whose slot is refilled below.
    if (k + S - 2 < nk) {
      if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER_WAVE) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_WAVE) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (k + S - 1 < nk) issue(k + S - 1, (k + S - 1) % S);
    const char* st = smem + (k % S) * STAGE;
    f32x4 a[MT], b[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) a[i] = *reinterpret_cast<const f32x4*>(st + a_off + i * 16 * 64);
#pragma unroll
    for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const f32x4*>(st + b_off + j * 16 * 64);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
  }

#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + j * 16 + l16;
    if (n >= p.Cout) continue;
    const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wid * 16 * MT + i * 16 + q * 4 + r;
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

template <int MT, int NT, int S>
hipError_t launch_dma(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_dma_f32<MT, NT, S>), dim3(mt * nt), dim3(256), 0, s, p, nt);
  return hipGetLastError();
}

template <int MT, int NT, int WM, int WN, int BK, bool SMALLC>
hipError_t launch_cfg(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_igemm_f32<MT, NT, WM, WN, BK, SMALLC>), dim3(mt * nt), dim3(64 * WM * WN), 0, s, p, nt);
  return hipGetLastError();
}

}  // namespace

// Tile choice per launch: among (MT, NT) with 16*NT dividing Cout, take the largest tile
// (MT*NT, ties -> larger MT: fewer re-reads of the weights) that still gives >= 3 blocks per CU;
// if none does, the smallest tile (most blocks). force_nt > 0 restricts NT (A/B experiments).
void conv_pick_tile(int M, int cout_p, int force_nt, int* mt_out, int* bn_out) {
  // Measured (round 1, 30 clips of 32x112x112): BM = 128 (mt = 2) beats 64 and 256 on every
  // layer -- 256 halves occupancy (LDS + accumulators), 64 doubles the weight re-reads of the
  // small-M layer4 convs -- and the widest N tile wins (the im2col A tile is read once).
  const int n16 = cout_p / 16;
  int nt = 3;
  for (int c : {9, 8, 6, 5, 4, 3})
    if (n16 % c == 0 && (force_nt <= 0 || c == force_nt)) {
      nt = c;
      break;
    }
  (void)M;
  *mt_out = 2;
  *bn_out = 16 * nt;
}

#define DMA_CASES(MT)                                  \
  switch (bn) {                                        \
    case 48: return launch_dma<MT, 3, 3>(p, s);        \
    case 64: return launch_dma<MT, 4, 3>(p, s);        \
    case 80: return launch_dma<MT, 5, 3>(p, s);        \
    case 96: return launch_dma<MT, 6, 3>(p, s);        \
    case 128: return launch_dma<MT, 8, 3>(p, s);       \
    case 144: return launch_dma<MT, 9, 3>(p, s);       \
  }

hipError_t launch_conv(const ConvParams& p, int mt, int bn, hipStream_t s) {
  if (p.Cin % 16 != 0) return launch_cfg<2, 3, 4, 1, 16, true>(p, s);  // stem: 3 (padded 4) channels
  if (mt == 4) {
    if (bn == 48) return launch_dma<4, 3, 3>(p, s);
    if (bn == 64) return launch_dma<4, 4, 3>(p, s);
  } else if (mt == 2) {
    DMA_CASES(2)
  } else if (mt == 1) {
    DMA_CASES(1)
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
