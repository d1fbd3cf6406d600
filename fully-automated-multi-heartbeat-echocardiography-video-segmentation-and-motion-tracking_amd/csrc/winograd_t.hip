// Fused 1-D Winograd F(4,3) along time for the stride-1 3x1x1 temporal convs of R(2+1)D-18 (fp32).
//
// Reference op: the Conv2Plus1D temporal conv3d(kernel (3,1,1), stride 1, padding (1,0,0)) + BN(eval)
// (+ residual) + ReLU of torchvision's r2plus1d_18, and the stem's second conv (called from
// src/model/R2plus1D_18_MotionNet.py:29-37).
//
//   y[4 frames] = A^T [ sum_ci U_ci (.) V_ci ],   U = G g (host, double, 6 values per 3 taps),
//                                                V = B^T d (6 input frames)
//
// 6 multiplies per 4 outputs and input channel instead of 12: the 6 transform elements are 6
// independent GEMMs M_e[tile][co] = sum_ci V_e[tile][ci] U_e[ci][co] on exact-fp32
// v_mfma_f32_16x16x4_f32. Interpolation points 0, +-1, +-2, inf.
//
// Block = 6 waves (wave e owns transform element e) x 64 tiles (4 frames at one pixel) x 64 output
// channels; 2 blocks per CU. Per chunk of 8 input channels:
//  * raw input (64 tiles x 6 frames x 32 B = 12 KB, [frame][tile][8 ci]) and U (6 e x 64 co x 32 B
//    = 12 KB, [e][co][8 ci]) arrive by LDS-DMA into 2-deep rings (wave e fetches its own U_e);
//  * all threads transform (tile, channel) columns into V (12 KB, [e][tile][8 ci], double-buffered);
//    the transform of chunk k+1 overlaps the MFMAs of chunk k; one barrier per chunk;
//  * 2 K steps x 4 m tiles x 4 n tiles = 32 MFMAs per chunk and wave.
// Epilogue: two 32-channel passes through LDS; each thread applies A^T to one (tile, channel) pair
// and writes 4 frames with bias, residual and ReLU.
#include <stdlib.h>

#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BT = 64;                   // tiles per block
constexpr int BN = 64;                   // output channels per block
constexpr int NTHR = 384;                // 6 waves
constexpr int RAW_BYTES = 6 * BT * 32;   // 12 KB
constexpr int V_BYTES = 6 * BT * 32;     // 12 KB
constexpr int U_BYTES = 6 * BN * 32;     // 12 KB
constexpr int LDS_BYTES = 2 * (RAW_BYTES + V_BYTES + U_BYTES);  // 72 KB
constexpr int MS = 36;                   // epilogue: floats per tile row (32 channels + 16-B pad)

__device__ inline int xcd_swizzle_t(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// KO != 0 only in tools/convbench.hip (knock-out timing builds): bit 1 no transform, 2 no raw DMA,
// 4 no U DMA, 8 no epilogue, 16 no MFMA.
template <int KO = 0>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(3, 3))) void conv_winot(ConvParams p, int n_co,
                                                                                              int n_tiles) {
  extern __shared__ __align__(16) char smem[];
  char* raw = smem;
  char* vbuf = smem + 2 * RAW_BYTES;
  char* ubuf = vbuf + 2 * V_BYTES;

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // = transform element e
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_t(blockIdx.x, gridDim.x);
  const int tb = blk / n_co, cb = blk - tb * n_co;
  const int t0 = tb * BT;
  const int T = p.To, HW = p.Ho * p.Wo, C = p.Cin, CO = p.Cout;
  const int TT = T >> 2;
  const int nchunk = C >> 3;

  // ---- raw DMA: 12 instructions per chunk, 2 per wave; slot s = I*64 + lane -> (frame, tile, half)
  int d_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int s = (wid * 2 + j) * 64 + lane;
    const int f = s >> 7, rem = s & 127, tl = rem >> 1, half = rem & 1;
    const int tg = t0 + tl;
    int off = -1;
    if (tg < n_tiles) {
      const int nt_ = tg / HW, pix = tg - nt_ * HW;
      const int n = nt_ / TT, tau = nt_ - n * TT;
      const int t = 4 * tau - 1 + f;
      if ((unsigned)t < (unsigned)T) off = ((n * T + t) * HW + pix) * C + half * 4;
    }
    d_off[j] = off;
  }
  // Past-the-end chunks fetch the zero block (or chunk 0 of U) into a free slot: every chunk issues
  // exactly 2 raw + 2 U DMAs per wave, so the counted waits below are exact.
  auto issue_raw = [&](int k, int buf) __attribute__((always_inline)) {
    if constexpr (KO & 2) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const void* src = (k < nchunk && d_off[j] >= 0) ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      char* dst = raw + buf * RAW_BYTES + (wid * 2 + j) * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  // U_e for chunk k: 2 KB at U + ((k*6 + e)*n_co + cb)*512 floats
  const float* ub = U + ((size_t)wid * n_co + cb) * 512 + lane * 4;
  auto issue_u = [&](int k, int buf) __attribute__((always_inline)) {
    if constexpr (KO & 4) return;
    const int kk = k < nchunk ? k : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const void* src = (const void*)(ub + (size_t)kk * 6 * n_co * 512 + j * 256);
      char* dst = ubuf + buf * U_BYTES + wid * 2048 + j * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  // ---- transform: (tile, channel) columns p = tid, tid + 384 (< 512)
  auto transform = [&](int buf) __attribute__((always_inline)) {
    if constexpr (KO & 1) return;
    const float* rb = reinterpret_cast<const float*>(raw + buf * RAW_BYTES);
    float* vb = reinterpret_cast<float*>(vbuf + buf * V_BYTES);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pr = tid + NTHR * h;
      if (pr < BT * 8) {
        float d[6];
#pragma unroll
        for (int f = 0; f < 6; ++f) d[f] = rb[f * (BT * 8) + pr];
        const float e1 = d[3] + d[4], e2 = d[1] + d[2], e3 = d[4] - d[3], e4 = d[1] - d[2];
        float* o = vb + pr;
        o[0 * BT * 8] = 4.f * d[0] - 5.f * d[2] + d[4];
        o[1 * BT * 8] = e1 - 4.f * e2;
        o[2 * BT * 8] = e3 + 4.f * e4;
        o[3 * BT * 8] = (d[4] - d[2]) + 2.f * (d[3] - d[1]);
        o[4 * BT * 8] = (d[4] - d[2]) - 2.f * (d[3] - d[1]);
        o[5 * BT * 8] = 4.f * d[1] - 5.f * d[3] + d[5];
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Chunk k: raw(k+2) is fetched at its start, U(k+2) at its end (the U slot is read until then);
  // at the top of chunk k, raw(k+1) and U(k) must have landed: only U(k+1)'s 2 DMAs are newer.
  issue_raw(0, 0);  // (the sched_barriers pin the issue order the counted vmcnt relies on)
  __builtin_amdgcn_sched_barrier(0);
  issue_u(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  issue_u(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | 6);  // vmcnt(6): raw(0) landed
  __builtin_amdgcn_s_barrier();
  transform(0);

  const int a_off = (l16 * 8 + 2 * q) * 4;  // byte offset of the lane's (tile l16, ci 2q..2q+1) pair
  for (int k = 0; k < nchunk; ++k) {
    __builtin_amdgcn_s_waitcnt(0x0070 | 2);  // vmcnt(2) lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // also: V(k) complete, everyone done with V(k-1) and raw(k)
    __builtin_amdgcn_sched_barrier(0);
    issue_raw(k + 2, k & 1);
    __builtin_amdgcn_sched_barrier(0);
    if (k + 1 < nchunk) transform((k + 1) & 1);
    const char* vb = vbuf + (k & 1) * V_BYTES + wid * (BT * 32) + a_off;
    const char* bb = ubuf + (k & 1) * U_BYTES + wid * 2048 + a_off;
    f32x2 a[4], b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) a[m] = *reinterpret_cast<const f32x2*>(vb + m * 16 * 32);
#pragma unroll
    for (int n = 0; n < 4; ++n) b[n] = *reinterpret_cast<const f32x2*>(bb + n * 16 * 32);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          if constexpr (KO & 16)
            acc[m][n][0] += a[m][s] * b[n][s];
          else
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s], b[n][s], acc[m][n], 0, 0, 0);
        }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of its U(k) slot are done
    __builtin_amdgcn_sched_barrier(0);
    issue_u(k + 2, k & 1);  // the U slot is private to the wave (its own e)
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the past-the-end DMAs before LDS is reused

  if constexpr ((KO & 8) != 0) {
    float sink = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) sink += acc[m][n][0] + acc[m][n][3];
    if (sink == 1.2345f) reinterpret_cast<float*>(p.y)[tid] = sink;
    return;
  }
  // ---- epilogue: y[4 frames] = A^T M, two passes of 32 channels through LDS. Unit = (tile, 4
  // consecutive channels): 16-B bias / residual loads and 16-B stores; each thread's global loads
  // are issued before the LDS exchange (res may alias y: no load waits behind a store).
  float* ms = reinterpret_cast<float*>(smem);
  constexpr int UNITS = BT * 8, UPT = (UNITS + NTHR - 1) / NTHR;
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  const size_t fstride = (size_t)HW * CO;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    size_t o0[UPT];
    bool ok[UPT];
    f32x4 rv[UPT][4], bv[UPT];
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int un = tid + NTHR * u;
      const int tl = un >> 3, cq = un & 7;
      const int tg = t0 + tl;
      ok[u] = un < UNITS && tg < n_tiles;
      const int tgc = ok[u] ? tg : 0;
      const int nt_ = tgc / HW, pix = tgc - nt_ * HW;
      const int n = nt_ / TT, tau = nt_ - n * TT;
      const int co = cb * BN + pass * 32 + 4 * cq;
      o0[u] = ((size_t)(n * T + 4 * tau) * HW + pix) * CO + co;
      bv[u] = (p.bias && ok[u]) ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a2 = 0; a2 < 4; ++a2)
        rv[u][a2] = (res && ok[u]) ? *reinterpret_cast<const f32x4*>(res + o0[u] + a2 * fstride)
                                   : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ms[(wid * BT + m * 16 + 4 * q + r) * MS + n2 * 16 + l16] = acc[m][2 * pass + n2][r];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      if (!ok[u]) continue;
      const int un = tid + NTHR * u;
      const int tl = un >> 3, cq = un & 7;
      f32x4 mm[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) mm[e] = *reinterpret_cast<const f32x4*>(ms + (e * BT + tl) * MS + 4 * cq);
      const f32x4 s12 = mm[1] + mm[2], d12 = mm[1] - mm[2], s34 = mm[3] + mm[4], d34 = mm[3] - mm[4];
      f32x4 yv[4];
      yv[0] = mm[0] + s12 + s34;
      yv[1] = d12 + 2.f * d34;
      yv[2] = s12 + 4.f * s34;
      yv[3] = d12 + 8.f * d34 + mm[5];
#pragma unroll
      for (int a2 = 0; a2 < 4; ++a2) {
        f32x4 v = yv[a2] + bv[u] + rv[u][a2];
        if (p.relu) {
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
        }
        *reinterpret_cast<f32x4*>(yout + o0[u] + a2 * fstride) = v;
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// conv_winot2: the same op for the large temporal convs (layer1 / stem at 32x112x112: 56x56 maps),
// re-blocked for MI355X's 4 SIMDs: 12 waves (3 per SIMD, one block per CU -- the 6-wave block
// above puts 2 waves on two SIMDs and 1 on the others, and its barrier makes the light SIMDs idle).
// Wave w owns transform element e = w % 6 for output-channel half nh = w / 6 (32 channels);
// block = 96 tiles x 64 channels (768 threads transform 96 x 8 (tile, channel) columns: one each).
// Rings: raw 3 (raw(k+3) is fetched at chunk k), U 2 (each wave fetches exactly the U_e half it
// reads), V 2. U and V rows carry a 16-B-slot swizzle (slot ^= (row >> 3) & 1) so the B / A
// operand ds_read_b64s are conflict-free. The transform of chunk k+1 is split around chunk k's
// MFMAs (reads first, arithmetic + V stores in their issue gaps).
constexpr int T2_BT = 96;
constexpr int T2_NTHR = 768;
constexpr int T2_RAW = 6 * T2_BT * 32;  // 18 KB: [frame][tile][8 ci]
constexpr int T2_V = 6 * T2_BT * 32;    // 18 KB: [e][tile][8 ci] (swizzled)
constexpr int T2_U = 6 * 64 * 32;       // 12 KB: [e][co][8 ci] (swizzled)
constexpr int T2_RAW_INSTR = T2_RAW / 1024;  // 18
constexpr int T2_LDS = 3 * T2_RAW + 2 * T2_U + 2 * T2_V;  // 114 KB
constexpr int T2_MS = 36;
static_assert(6 * T2_BT * T2_MS * 4 <= T2_LDS, "epilogue exchange");

__device__ inline int swz(int row, int ci) { return row * 8 + ((((ci >> 2) ^ (row >> 3)) & 1) << 2) + (ci & 3); }

template <int KO = 0>
__global__ __launch_bounds__(T2_NTHR) void conv_winot2(ConvParams p, int n_co, int n_tiles) {
  extern __shared__ __align__(16) char smem[];
  char* raw = smem;
  char* ubuf = raw + 3 * T2_RAW;
  char* vbuf = ubuf + 2 * T2_U;

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int e = wid % 6, nh = wid / 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_t(blockIdx.x, gridDim.x);
  const int tb = blk / n_co, cb = blk - tb * n_co;
  const int t0 = tb * T2_BT;
  const int T = p.To, HW = p.Ho * p.Wo, C = p.Cin, CO = p.Cout;
  const int TT = T >> 2;
  const int nchunk = C >> 3;
  const bool two_raw = wid + 12 < T2_RAW_INSTR;

  // raw DMA: instruction I in {wid, wid + 12} fills slots s = I*64 + lane -> (frame, tile, half)
  int d_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int s = (wid + 12 * j) * 64 + lane;
    const int f = s / (T2_BT * 2), rem = s - f * (T2_BT * 2), tl = rem >> 1, half = rem & 1;
    const int tg = t0 + tl;
    int off = -1;
    if (s < T2_RAW_INSTR * 64 && tg < n_tiles) {
      const int nt_ = tg / HW, pix = tg - nt_ * HW;
      const int n = nt_ / TT, tau = nt_ - n * TT;
      const int t = 4 * tau - 1 + f;
      if ((unsigned)t < (unsigned)T) off = ((n * T + t) * HW + pix) * C + half * 4;
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
    if constexpr (KO & 2) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && !two_raw) break;
      const void* src = (k < nchunk && d_off[j] >= 0) ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(raw + stage * T2_RAW +
                                                                                 (wid + 12 * j) * 1024),
                                       16, 0, 0);
    }
  };
  // U DMA: this wave's 1 KB = U_e rows co = 32 nh .. +32 (lane -> LDS slot (co, h'), global slot h =
  // h' ^ ((co >> 3) & 1))
  const int u_co = 32 * nh + (lane >> 1), u_h = (lane & 1) ^ ((u_co >> 3) & 1);
  const float* u_src = U + ((size_t)e * n_co + cb) * 512 + u_co * 8 + u_h * 4;
  auto issue_u = [&](int k, int stage) __attribute__((always_inline)) {
    if constexpr (KO & 4) return;
    const size_t kk = k < nchunk ? k : 0;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(u_src + kk * 6 * n_co * 512),
                                     (__attribute__((address_space(3))) void*)(ubuf + stage * T2_U + e * 2048 +
                                                                               nh * 1024 + lane * 16),
                                     16, 0, 0);
  };
  // transform: thread = (tile tid >> 3, channel tid & 7)
  const int tr_tile = tid >> 3, tr_ci = tid & 7;
  const int tr_v = swz(tr_tile, tr_ci);
  auto transform_read = [&](int stage, float (&d)[6]) __attribute__((always_inline)) {
    if constexpr (KO & 1) {
#pragma unroll
      for (int f = 0; f < 6; ++f) d[f] = (float)(stage + f);
      return;
    }
    const float* rb = reinterpret_cast<const float*>(raw + stage * T2_RAW) + tid;
#pragma unroll
    for (int f = 0; f < 6; ++f) d[f] = rb[f * (T2_BT * 8)];
  };
  auto transform_write = [&](const float (&d)[6], int stage) __attribute__((always_inline)) {
    if constexpr (KO & 1) return;
    float* o = reinterpret_cast<float*>(vbuf + stage * T2_V) + tr_v;
    const float e1 = d[3] + d[4], e2 = d[1] + d[2], e3 = d[4] - d[3], e4 = d[1] - d[2];
    o[0 * T2_BT * 8] = 4.f * d[0] - 5.f * d[2] + d[4];
    o[1 * T2_BT * 8] = e1 - 4.f * e2;
    o[2 * T2_BT * 8] = e3 + 4.f * e4;
    o[3 * T2_BT * 8] = (d[4] - d[2]) + 2.f * (d[3] - d[1]);
    o[4 * T2_BT * 8] = (d[4] - d[2]) - 2.f * (d[3] - d[1]);
    o[5 * T2_BT * 8] = 4.f * d[1] - 5.f * d[3] + d[5];
  };

  f32x4 acc[6][2];
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: raw(0), U(0), raw(1), U(1), raw(2); transform(0)
  issue_raw(0, 0);  // (the sched_barriers pin the issue order the counted vmcnt relies on)
  __builtin_amdgcn_sched_barrier(0);
  issue_u(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  issue_u(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(2, 2);
  __builtin_amdgcn_sched_barrier(0);
  if (two_raw)
    __builtin_amdgcn_s_waitcnt(0x0F70 | 6);  // vmcnt(2 + 2*2): raw(0) landed
  else
    __builtin_amdgcn_s_waitcnt(0x0F70 | 4);
  __builtin_amdgcn_s_barrier();
  {
    float d[6];
    transform_read(0, d);
    transform_write(d, 0);
  }

  // lane operand offsets (floats) inside an e slice: A rows = tiles 16m + l16, B rows = channels
  const int a_row = l16, b_row = 32 * nh + l16;
  for (int k = 0; k < nchunk; ++k) {
    if (two_raw)
      __builtin_amdgcn_s_waitcnt(0x0070 | 3);  // vmcnt(nraw + 1): raw(k+1), U(k) landed; lgkmcnt(0)
    else
      __builtin_amdgcn_s_waitcnt(0x0070 | 2);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const float* vb = reinterpret_cast<const float*>(vbuf + (k & 1) * T2_V) + e * (T2_BT * 8);
    const float* ub = reinterpret_cast<const float*>(ubuf + (k & 1) * T2_U) + e * 512;
    f32x2 a[6], b[2];
#pragma unroll
    for (int m = 0; m < 6; ++m) a[m] = *reinterpret_cast<const f32x2*>(vb + swz(16 * m + a_row, 2 * q));
#pragma unroll
    for (int n = 0; n < 2; ++n) b[n] = *reinterpret_cast<const f32x2*>(ub + swz(16 * n + b_row, 2 * q));
    float d[6];
    transform_read((k + 1) % 3, d);
    issue_raw(k + 3, k % 3);  // after this chunk's LDS reads: rides in the first MFMA gaps
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int m = 0; m < 6; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if constexpr (KO & 16)
            acc[m][n][0] += a[m][s2] * b[n][s2];
          else
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s2], b[n][s2], acc[m][n], 0, 0, 0);
        }
    transform_write(d, (k + 1) & 1);
    if constexpr (KO == 0) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (raw LDS-DMA)
      }
#pragma unroll
      for (int g = 0; g < 6; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
      }
#pragma unroll
      for (int g = 0; g < 6; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of its U(k) half are done
    __builtin_amdgcn_sched_barrier(0);
    issue_u(k + 2, k & 1);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the past-the-end DMAs before LDS is reused

  if constexpr ((KO & 8) != 0) {
    float sink = 0.f;
#pragma unroll
    for (int m = 0; m < 6; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) sink += acc[m][n][0] + acc[m][n][3];
    if (sink == 1.2345f) reinterpret_cast<float*>(p.y)[tid] = sink;
    return;
  }
  // epilogue: two passes (channel halves); in pass h the waves with nh == h publish M through LDS,
  // then every thread applies A^T to one (tile, 4-channel) unit and writes 4 frames.
  float* ms = reinterpret_cast<float*>(smem);
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  const size_t fstride = (size_t)HW * CO;
  const int ut = tid >> 3, cq = tid & 7;
  const int tg = t0 + ut;
  const bool ok = tg < n_tiles;
  size_t o0;
  {
    const int tgc = ok ? tg : 0;
    const int nt_ = tgc / HW, pix = tgc - nt_ * HW;
    const int n = nt_ / TT, tau = nt_ - n * TT;
    o0 = ((size_t)(n * T + 4 * tau) * HW + pix) * CO + cb * 64 + 4 * cq;
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const size_t o = o0 + pass * 32;
    const f32x4 bv = (p.bias && ok) ? *reinterpret_cast<const f32x4*>(p.bias + cb * 64 + pass * 32 + 4 * cq)
                                    : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 rv[4];
#pragma unroll
    for (int a2 = 0; a2 < 4; ++a2)
      rv[a2] = (res && ok) ? *reinterpret_cast<const f32x4*>(res + o + a2 * fstride) : f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    if (nh == pass) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int m = 0; m < 6; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ms[(e * T2_BT + m * 16 + 4 * q + r) * T2_MS + n * 16 + l16] = acc[m][n][r];
    }
    __syncthreads();
    if (ok) {
      f32x4 mm[6];
#pragma unroll
      for (int e2 = 0; e2 < 6; ++e2) mm[e2] = *reinterpret_cast<const f32x4*>(ms + (e2 * T2_BT + ut) * T2_MS + 4 * cq);
      const f32x4 s12 = mm[1] + mm[2], d12 = mm[1] - mm[2], s34 = mm[3] + mm[4], d34 = mm[3] - mm[4];
      f32x4 yv[4];
      yv[0] = mm[0] + s12 + s34;
      yv[1] = d12 + 2.f * d34;
      yv[2] = s12 + 4.f * s34;
      yv[3] = d12 + 8.f * d34 + mm[5];
#pragma unroll
      for (int a2 = 0; a2 < 4; ++a2) {
        f32x4 v = yv[a2] + bv + rv[a2];
        if (p.relu) {
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
        }
        *reinterpret_cast<f32x4*>(yout + o + a2 * fstride) = v;
      }
    }
  }
}

template <int KO>
hipError_t winot2_launch(const ConvParams& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot2<KO>, hipFuncAttributeMaxDynamicSharedMemorySize, T2_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
  const int n_co = p.Cout / 64;
  hipLaunchKernelGGL(conv_winot2<KO>, dim3(((n_tiles + T2_BT - 1) / T2_BT) * n_co), dim3(T2_NTHR), T2_LDS, s, p, n_co,
                     n_tiles);
  return hipGetLastError();
}

}  // namespace

bool winot_supported(const ConvParams& p) {
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && p.KT == 3 && p.KH == 1 && p.KW == 1 && p.st == 1 &&
         p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 0 && p.pw == 0 && p.Cin % 8 == 0 && p.Cout % BN == 0 &&
         p.To == p.Ti && p.Ti % 4 == 0 && p.Ho == p.Hi && p.Wo == p.Wi &&
         (size_t)p.N * p.Ti * p.Hi * p.Wi * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31);
}

// U: [Cin/8][6][Cout/64][64][8] transformed weights (winot_transform_weights).
hipError_t launch_winot(const ConvParams& p, hipStream_t s) {
  if (!winot_supported(p)) return hipErrorInvalidValue;
  const bool no_t2 = getenv("CLASFV_NO_WINOT2") != nullptr;  // A/B switch (tests)
  // the 12-wave kernel wins from layer3 (490 blocks of 96 tiles) up; below one block per CU the
  // 2-blocks-per-CU 64-tile kernel keeps more of the chip busy
  if (!no_t2 && (size_t)p.N * (p.Ti / 4) * p.Hi * p.Wi / T2_BT * (p.Cout / 64) >= 256) return winot2_launch<0>(p, s);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot<0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
  const int n_co = p.Cout / BN;
  const int nb = (n_tiles + BT - 1) / BT;
  hipLaunchKernelGGL(conv_winot<0>, dim3(nb * n_co), dim3(NTHR), LDS_BYTES, s, p, n_co, n_tiles);
  return hipGetLastError();
}

#ifdef CLASFV_KNOCKOUTS
template <int KO>
static hipError_t winot_ko(const ConvParams& p, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute((const void*)conv_winot<KO>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  if (e != hipSuccess) return e;
  const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
  const int n_co = p.Cout / BN;
  hipLaunchKernelGGL(conv_winot<KO>, dim3(((n_tiles + BT - 1) / BT) * n_co), dim3(NTHR), LDS_BYTES, s, p, n_co, n_tiles);
  return hipGetLastError();
}
hipError_t launch_winot_ko(const ConvParams& p, hipStream_t s, int ko) {
  switch (ko) {
    case 0: return winot_ko<0>(p, s);
    case 1: return winot_ko<1>(p, s);
    case 2: return winot_ko<2>(p, s);
    case 4: return winot_ko<4>(p, s);
    case 8: return winot_ko<8>(p, s);
    case 16: return winot_ko<16>(p, s);
    case 6: return winot_ko<6>(p, s);
    case 7: return winot_ko<7>(p, s);
    case 15: return winot_ko<15>(p, s);
    case 100: return winot2_launch<0>(p, s);
    case 101: return winot2_launch<1>(p, s);
    case 102: return winot2_launch<2>(p, s);
    case 104: return winot2_launch<4>(p, s);
    case 108: return winot2_launch<8>(p, s);
    case 115: return winot2_launch<15>(p, s);
  }
  return hipErrorInvalidValue;
}
#endif

// Host: U[c/8][e][o/64][o%64][c%8] = (G g_{o,c})[e] in double, g = folded 3-tap temporal kernel.
void winot_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  const int ncb = cout_p / BN;
  for (size_t i = 0; i < (size_t)6 * cin_p * cout_p; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* g = w + ((size_t)o * cin + c) * 3;
      for (int e = 0; e < 6; ++e) {
        const double u = G[e][0] * g[0] + G[e][1] * g[1] + G[e][2] * g[2];
        U[((((size_t)(c / 8) * 6 + e) * ncb + o / BN) * BN + o % BN) * 8 + c % 8] = (float)u;
      }
    }
}
