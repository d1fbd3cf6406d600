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
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s], b[n][s], acc[m][n], 0, 0, 0);
        }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of its U(k) slot are done
    __builtin_amdgcn_sched_barrier(0);
    issue_u(k + 2, k & 1);  // the U slot is private to the wave (its own e)
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the past-the-end DMAs before LDS is reused

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
    const float* rb = reinterpret_cast<const float*>(raw + stage * T2_RAW) + tid;
#pragma unroll
    for (int f = 0; f < 6; ++f) d[f] = rb[f * (T2_BT * 8)];
  };
  auto transform_write = [&](const float (&d)[6], int stage) __attribute__((always_inline)) {
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
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s2], b[n][s2], acc[m][n], 0, 0, 0);
        }
    transform_write(d, (k + 1) & 1);
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
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of its U(k) half are done
    __builtin_amdgcn_sched_barrier(0);
    issue_u(k + 2, k & 1);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the past-the-end DMAs before LDS is reused

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

hipError_t winot2_launch(const ConvParams& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot2, hipFuncAttributeMaxDynamicSharedMemorySize, T2_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
  const int n_co = p.Cout / 64;
  hipLaunchKernelGGL(conv_winot2, dim3(((n_tiles + T2_BT - 1) / T2_BT) * n_co), dim3(T2_NTHR), T2_LDS, s, p, n_co,
                     n_tiles);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// conv_winot3: the same op with a rolling temporal halo and the output transform in registers.
//  * A block owns P pixel columns (a column = one pixel of one clip; columns of consecutive clips
//    are contiguous, so small maps do not leave ragged blocks) x a segment of TS temporal tiles
//    (4*TS output frames) x 64 output channels. Its raw input per 8-channel chunk is the segment's
//    4*TS + 2 frames of the P columns, fetched ONCE: adjacent tiles share their 2-frame halo
//    (34 frames for 32 outputs at TS = 8 instead of 48: the 6-in / 4-out over-fetch of per-tile
//    windows drops from 1.5x to 1.06x).
//  * Operands are swapped relative to conv_winot: D^T = U^T V^T, so an accumulator lane holds 4
//    CONSECUTIVE output channels of one tile; each wave holds all 6 transform elements of its tiles,
//    so y = A^T M is applied in registers and written with 16-B stores -- no LDS exchange, no
//    epilogue barrier. Same products, same channel order per MFMA (k = 2q + s2), same fp32 chain:
//    bit-identical to conv_winot / conv_winot2.
//  * Each lane transforms its own (tile, channel pair) straight from the raw frames in LDS into
//    MFMA B operands (no V round trip through LDS); U operands come from L2 into registers one
//    chunk ahead. Per chunk and wave: 10-12 ds_read_b64, 48 MFMAs (6 e x 2 tiles x 2 co tiles x
//    2 k-steps); one barrier per chunk (3-stage raw ring).
// Wave w: co half h = w & 1 (32 channels), tile pair pr = w >> 1 (m-tiles 2pr, 2pr+1). m-tile j =
// (column group j / TS of 16 columns, tile j % TS of the segment). NW waves -> NW m-tiles.
// Raw LDS image: [local frame lf][column c][16-B half], the half index XOR ((c >> 3) & 1) so the
// 16 columns x 4 lane groups of a ds_read_b64 hit 64 distinct banks.
template <int NW, int TS>
struct T3 {
  static constexpr int P = 16 * NW / TS;             // columns per block
  static constexpr int NF = 4 * TS + 2;              // raw frames per segment
  static constexpr int SLOTS = NF * P * 2;           // 16-B slots per chunk
  static constexpr int NI = (SLOTS + 63) / 64;       // DMA wave-instructions per chunk
  static constexpr int DPW = (NI + NW - 1) / NW;     // per wave, waves w < NI % NW (or all): DPW, else DPW-1
  static constexpr int DLO = NI / NW;                // DMAs of the waves that issue fewer
  static constexpr int STAGE = NI * 1024;
  static constexpr int LDS = 3 * STAGE;
  static_assert(P >= 16 && P % 16 == 0, "at least one 16-column group per block");
};

template <int NW, int TS>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_winot3(ConvParams p, int n_co,
                                                                                                int n_seg, int n_cols) {
  using G = T3<NW, TS>;
  extern __shared__ __align__(16) char smem[];

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w_alt);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  const bool full = (G::NI % NW == 0) || wid < G::NI % NW;  // issues DPW DMAs per chunk (else DLO)
  const int blk = xcd_swizzle_t(blockIdx.x, gridDim.x);
  const int co_blk = blk % n_co, rest = blk / n_co;
  const int seg = rest % n_seg, cb = rest / n_seg;
  const int col0 = cb * G::P, co0 = co_blk * 64;
  const int T = p.To, HW = p.Ho * p.Wo, C = p.Cin, CO = p.Cout;
  const int t_seg = seg * 4 * TS;  // first output frame of the segment
  const int nchunk = C >> 3;

  // raw DMA slots: instruction wid + NW*j, lane -> slot s -> (lf, column c, stored half hs). Every
  // source is a valid address: frames outside [0, T) and columns past the end are clamped (their
  // values are zeroed in registers / their outputs discarded) and the slots past SLOTS re-read
  // element 0 into the sink. So the issue is saddr (chunk base, scalar) + a fixed 32-bit voffset.
  unsigned d_off[G::DPW];
#pragma unroll
  for (int j = 0; j < G::DPW; ++j) {
    const int s = (wid + NW * j) * 64 + lane;
    unsigned off = 0;
    if (s < G::SLOTS) {
      const int lf = s / (2 * G::P), rem = s - lf * (2 * G::P), c = rem >> 1;
      const int half = (rem & 1) ^ ((c >> 3) & 1);
      int gc = col0 + c, t = t_seg - 1 + lf;
      gc = gc < n_cols ? gc : n_cols - 1;
      t = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const int n = gc / HW, pix = gc - n * HW;
      off = (unsigned)(((n * T + t) * HW + pix) * C + half * 4) * 4u;  // bytes (< 2^31, host-checked)
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
    const char* xk = reinterpret_cast<const char*>(x + k * 8);
#pragma unroll
    for (int j = 0; j < G::DPW; ++j) {
      if (j == G::DLO && !full) break;  // wave-uniform
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xk + d_off[j]),
                                       (__attribute__((address_space(3))) void*)(smem + stage * G::STAGE +
                                                                                 (wid + NW * j) * 1024),
                                       16, 0, 0);
    }
  };
  // U (A operand): lane (co = l16 of n tile nt, channels 2q, 2q+1) of element e, chunk k:
  // U[((k*6 + e)*CO + co)*8 + 2q], two floats
  const int h = wid & 1, pr = wid >> 1;
  // U (A operand) in the winot3 layout [k][e pair][co][q][e & 1][2 ci] (winot3_transform_weights):
  // one 16-B load per (e pair, n tile) gives the lane's channels 2q, 2q+1 of co for both elements
  const unsigned u_lane = (unsigned)(((co0 + 32 * h + l16) * 4 + q) * 4) * 4u;  // bytes
  auto load_u = [&](int k, f32x2 (&u)[6][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int ep = 0; ep < 3; ++ep)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const char* ue = reinterpret_cast<const char*>(U + ((size_t)k * 3 + ep) * CO * 16 + nt * 256);
        const f32x4 v = *reinterpret_cast<const f32x4*>(ue + u_lane);
        u[2 * ep][nt] = f32x2{v[0], v[1]};
        u[2 * ep + 1][nt] = f32x2{v[2], v[3]};
      }
  };
  // the lane's raw reads: tile column c = (m-tile group) * 16 + l16, channel pair q
  int rd_off[2];  // float offset of local frame 0 of each of the wave's two m-tiles
  bool pad_lo[2], pad_hi[2];  // the tile's first / last input frame lies outside [0, T): zero it
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int j = 2 * pr + m;
    const int c = (j / TS) * 16 + l16;
    const int slot = c * 2 + ((q >> 1) ^ ((c >> 3) & 1));
    rd_off[m] = (4 * (j % TS)) * (G::P * 8) + slot * 4 + (q & 1) * 2;
    const int t0 = t_seg + 4 * (j % TS);
    pad_lo[m] = t0 == 0;
    pad_hi[m] = t0 + 4 >= T;
  }

  f32x4 acc[6][2][2];
#pragma unroll
  for (int e = 0; e < 6; ++e)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[e][m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x2 ua[6][2], ubb[6][2];

  // prologue: U(0), raw(0), raw(1); chunk k issues U(k+1) loads, then raw(k+2) DMAs -- so at the top
  // of chunk k only raw(k+1)'s DPW DMAs may still be outstanding
  load_u(0, ua);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);

  // mode 2: U(k+1) + raw(k+2) follow (k + 2 < nchunk); 1: only U(k+1) (k == nchunk - 2); 0: last
  // chunk. Every call passes a literal mode: each inlined copy has straight-line, exact vmcnt waits.
  auto step = [&](int k, f32x2 (&uc)[6][2], f32x2 (&un)[6][2], int mode) __attribute__((always_inline)) {
    if (mode > 0) {  // vmcnt(own raw(k+1) DMAs) lgkmcnt(0): raw(k), U(k) landed
      if (full)
        __builtin_amdgcn_s_waitcnt(0x0070 | G::DPW);
      else
        __builtin_amdgcn_s_waitcnt(0x0070 | G::DLO);
    } else {
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave's raw(k) landed; everyone done with stage (k-1) % 3
    __builtin_amdgcn_sched_barrier(0);
    if (mode > 0) load_u(k + 1, un);
    __builtin_amdgcn_sched_barrier(0);
    if (mode > 1) issue_raw(k + 2, (k + 2) % 3);
    __builtin_amdgcn_sched_barrier(0);
    const float* rb = reinterpret_cast<const float*>(smem + (k % 3) * G::STAGE);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      f32x2 d[6];
#pragma unroll
      for (int f = 0; f < 6; ++f) d[f] = *reinterpret_cast<const f32x2*>(rb + rd_off[m] + f * (G::P * 8));
      if (pad_lo[m]) d[0] = f32x2{0.f, 0.f};
      if (pad_hi[m]) d[5] = f32x2{0.f, 0.f};
      f32x2 v[6];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const float d0 = d[0][s2], d1 = d[1][s2], d2 = d[2][s2], d3 = d[3][s2], d4 = d[4][s2], d5 = d[5][s2];
        const float e1 = d3 + d4, e2 = d1 + d2, e3 = d4 - d3, e4 = d1 - d2;
        v[0][s2] = 4.f * d0 - 5.f * d2 + d4;
        v[1][s2] = e1 - 4.f * e2;
        v[2][s2] = e3 + 4.f * e4;
        v[3][s2] = (d4 - d2) + 2.f * (d3 - d1);
        v[4][s2] = (d4 - d2) - 2.f * (d3 - d1);
        v[5][s2] = 4.f * d1 - 5.f * d3 + d5;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int e = 0; e < 6; ++e)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[e][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(uc[e][nt][s2], v[e][s2], acc[e][m][nt], 0, 0, 0);
    }
  };
  // nchunk is even (Cin % 16 == 0, host-checked): pairs of chunks, the last pair without prefetch
  int k = 0;
  for (; k + 4 <= nchunk; k += 2) {
    step(k, ua, ubb, 2);
    step(k + 1, ubb, ua, 2);
  }
  step(k, ua, ubb, 1);
  step(k + 1, ubb, ua, 0);

  // epilogue: y[a] = A^T M per (tile, 4 channels) in registers; 16-B residual loads and stores
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  const size_t fstride = (size_t)HW * CO;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int j = 2 * pr + m;
    const int gc = col0 + (j / TS) * 16 + l16;
    const bool ok = gc < n_cols;
    const int gcc = ok ? gc : 0;
    const int n = gcc / HW, pix = gcc - n * HW;
    const int t0 = t_seg + 4 * (j % TS);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int co = co0 + 32 * h + 16 * nt + 4 * q;
      const size_t o = ((size_t)(n * T + t0) * HW + pix) * CO + co;
      const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 rv[4];
#pragma unroll
      for (int a2 = 0; a2 < 4; ++a2)
        rv[a2] = (res && ok) ? *reinterpret_cast<const f32x4*>(res + o + a2 * fstride) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4* mm = &acc[0][m][nt];
      const f32x4 m0 = acc[0][m][nt], m1 = acc[1][m][nt], m2 = acc[2][m][nt], m3 = acc[3][m][nt],
                  m4 = acc[4][m][nt], m5 = acc[5][m][nt];
      (void)mm;
      const f32x4 s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
      f32x4 yv[4];
      yv[0] = m0 + s12 + s34;
      yv[1] = d12 + 2.f * d34;
      yv[2] = s12 + 4.f * s34;
      yv[3] = d12 + 8.f * d34 + m5;
      if (ok) {
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
}

template <int NW, int TS>
hipError_t winot3_launch(const ConvParams& p, hipStream_t s) {
  using G = T3<NW, TS>;
  static bool attr = false;
  if (!attr && G::LDS > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot3<NW, TS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int n_cols = p.N * p.Hi * p.Wi;
  const int n_seg = (p.Ti / 4) / TS;
  const int n_co = p.Cout / 64;
  const int nb = ((n_cols + G::P - 1) / G::P) * n_seg * n_co;
  hipLaunchKernelGGL((conv_winot3<NW, TS>), dim3(nb), dim3(64 * NW), G::LDS, s, p, n_co, n_seg, n_cols);
  return hipGetLastError();
}

// TS = temporal tiles per segment: the largest of 8 (NW = 8) / 4 (NW = 4) that divides T / 4.
template <int NW>
hipError_t winot3_dispatch(const ConvParams& p, hipStream_t s) {
  const int tt = p.Ti / 4;
  if (NW == 8 && tt % 8 == 0) return winot3_launch<NW, NW == 8 ? 8 : 4>(p, s);
  if (tt % 4 == 0) return winot3_launch<NW, 4>(p, s);
  if (tt % 2 == 0) return winot3_launch<NW, 2>(p, s);
  return winot3_launch<NW, 1>(p, s);
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
  // CLASFV_NO_WINOT2=1 (tests): always the 6-wave reference kernel; the three kernels compute the
  // same products in the same order (bit-identical outputs).
  const bool base_only = getenv("CLASFV_NO_WINOT2") != nullptr;
  // rolling-halo kernel for T >= 16 (measured: layer1/stem/layer2 maps at 30 clips and 64-frame
  // clips 3-20 % faster than conv_winot2, and 1.06x instead of 1.5x input fetch); at T = 8 the
  // 12-wave kernel is ahead (0.236 vs 0.249 ms on layer3), below one block per CU the 6-wave one
  if (!base_only && p.w_alt && p.Ti % 8 == 0 && p.Ti >= 16 && p.Cin % 16 == 0) return winot3_dispatch<4>(p, s);
  if (!base_only && (size_t)p.N * (p.Ti / 4) * p.Hi * p.Wi / T2_BT * (p.Cout / 64) >= 256) return winot2_launch(p, s);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
  const int n_co = p.Cout / BN;
  const int nb = (n_tiles + BT - 1) / BT;
  hipLaunchKernelGGL(conv_winot, dim3(nb * n_co), dim3(NTHR), LDS_BYTES, s, p, n_co, n_tiles);
  return hipGetLastError();
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: run one temporal kernel variant (0 conv_winot, 100 conv_winot2, 300 / 301
// conv_winot3 with 4 / 8 waves); timing and bit-identity comparisons only, not product code.
hipError_t launch_winot_ko(const ConvParams& p, hipStream_t s, int ko) {
  switch (ko) {
    case 0: {
      hipError_t e = hipFuncSetAttribute((const void*)conv_winot, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      if (e != hipSuccess) return e;
      const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
      hipLaunchKernelGGL(conv_winot, dim3(((n_tiles + BT - 1) / BT) * (p.Cout / BN)), dim3(NTHR), LDS_BYTES, s, p,
                         p.Cout / BN, n_tiles);
      return hipGetLastError();
    }
    case 100: return winot2_launch(p, s);
    case 300: return winot3_dispatch<4>(p, s);
    case 301: return winot3_dispatch<8>(p, s);
  }
  return hipErrorInvalidValue;
}
#endif

// Host: the conv_winot3 layout U3[c/8][e/2][o][(c%8)/2][e%2][c%2] of the same values.
void winot3_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  for (size_t i = 0; i < (size_t)6 * cin_p * cout_p; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* g = w + ((size_t)o * cin + c) * 3;
      for (int e = 0; e < 6; ++e) {
        const double u = G[e][0] * g[0] + G[e][1] * g[1] + G[e][2] * g[2];
        U[(((((size_t)(c / 8) * 3 + e / 2) * cout_p + o) * 4 + (c % 8) / 2) * 2 + e % 2) * 2 + c % 2] = (float)u;
      }
    }
}

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
