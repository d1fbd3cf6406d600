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
          for (int c = 0; c < 4; ++c) v[c] = relu1(v[c]);
        }
        *reinterpret_cast<f32x4*>(yout + o0[u] + a2 * fstride) = v;
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// conv_winot5: the same op for T % 8 == 0, re-blocked around three measured costs of the kernel
// above (tools/bench_winot.sh; 30 clips, layer1 144->64: 1.48 -> 1.04 ms, layer2 288->128: 0.68 ->
// 0.43 ms, bit-identical outputs):
//  * rolling temporal halo: a block owns P pixel columns (a column = one pixel of one clip; columns of
//    consecutive clips are contiguous, so small maps leave no ragged blocks) x a segment of TS
//    temporal tiles (4*TS output frames) x 64 output channels, and fetches the segment's 4*TS + 2
//    input frames ONCE per 8-channel chunk: adjacent tiles share their 2-frame halo (18 frames for
//    16 outputs instead of 24: 1.125x input fetch instead of 1.5x);
//  * U staged in LDS: each chunk's U slice for the block's 64 channels (12 KiB, conv_winot's U
//    layout) arrives by LDS-DMA with the raw frames and every wave reads its fragments with
//    conflict-free ds_read_b64 (16-B half index ^ ((co >> 3) & 1)) -- per-lane global U loads cost
//    ~20 % of the kernel in a register-operand variant;
//  * output transform in registers: operands swapped (D^T = U^T V^T), so an accumulator lane holds
//    4 consecutive output channels of one tile and each wave holds all 6 transform elements of its
//    tiles: y = A^T M, bias, residual and ReLU go straight to 16-B stores, no LDS exchange.
// Each lane transforms its own (tile column, channel pair) from the raw frames into MFMA B operands
// (no V round trip through LDS). A wave owns 2 tiles (adjacent in time: they share 2 of their 10
// frames) x 64 channels: 96 MFMAs per chunk and barrier; 2 LDS stages, 2 blocks per CU.
// TS = 1 (T = 4: one temporal tile, layer4 at 32-frame clips): a wave's 2 tiles are 2 column groups
// of the single tile row instead (6 frames each), in the same accumulation order.
template <int TS, int NT>
struct T5 {
  static constexpr int P = 16 * 8 / TS;          // columns per block
  static constexpr int NF = 4 * TS + 2;          // raw frames per chunk
  static constexpr int RAW_I = NF * P * 2 / 64;  // raw DMA wave-instructions per chunk
  static constexpr int CB = 16 * NT;             // output channels per block (and per wave)
  static constexpr int U_I = 6 * CB * 32 / 1024; // U: 6 e x CB co x 32 B
  static constexpr int NI = RAW_I + U_I;
  static constexpr int STAGE = NI * 1024;
  static constexpr int LDS = 2 * STAGE;
  static_assert(NF * P * 2 % 64 == 0, "whole DMA instructions");
};

// EPI: epilogue form, bit 0 = residual add, bit 1 = ReLU (compile-time, no per-element selects);
// bit 2 = split-K partial: the block sums input-channel chunks [k0, k1) of its split only and stores
// y = A^T M without bias, residual or ReLU to p.part[split] (launch_split_sum finishes).
template <int TS, int NT, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((EPI & 16384) ? 3 : 2, (EPI & 16384) ? 3 : 2))) void conv_winot5(ConvParams p, int n_co,
                                                                                             int n_seg, int n_cols,
                                                                                             FastDiv fd_hw) {
  using G = T5<TS, NT>;
  extern __shared__ __align__(16) char smem[];
  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  constexpr bool SPLIT = (EPI & 4) != 0;
  int blk = xcd_swizzle_t(blockIdx.x, gridDim.x);
  const int nb = gridDim.x / (SPLIT ? p.n_split : 1);
  const int split = SPLIT ? blk / nb : 0;
  blk -= split * nb;
  const int co_blk = blk % n_co, rest = blk / n_co;
  const int seg = rest % n_seg, cb = rest / n_seg;
  const int col0 = cb * G::P, co0 = co_blk * G::CB;
  const int T = p.To, HW = p.Ho * p.Wo, C = p.Cin, CO = p.Cout;
  const int t_seg = seg * 4 * TS;
  const int nchunk = C >> 3;
  const int k0 = SPLIT ? split * nchunk / p.n_split : 0;
  const int k1 = SPLIT ? (split + 1) * nchunk / p.n_split : nchunk;
  // input pixel stride and chunk stride (floats): channels-last, or 8-channel blocks (x_c8)
  const int cs = p.x_c8 ? 8 : C;
  const size_t kstride = p.x_c8 ? (size_t)p.N * T * HW * 8 : 8;
  constexpr int DMAX = (G::NI + 3) / 4;           // DMA instructions of waves 0 .. (NI % 4) - 1
  constexpr int DMIN = G::NI / 4;                 // ... of the others
  const bool more = (G::NI % 4 == 0) || wid < G::NI % 4;

  // DMA slots: instruction I = wid + 4j; I < RAW_I: raw frames, else U. Byte offsets relative to the
  // chunk's scalar base (x + 8k floats for raw, U + 6*CO*8*k floats for U); every source is valid.
  unsigned d_off[DMAX];
#pragma unroll
  for (int j = 0; j < DMAX; ++j) {
    const int I = wid + 4 * j;
    unsigned off = 0;
    if (I < G::RAW_I) {
      const int s = I * 64 + lane;
      const int lf = s / (2 * G::P), rem = s - lf * (2 * G::P), c = rem >> 1;
      const int half = (rem & 1) ^ ((c >> 3) & 1);
      int gc = col0 + c, t = t_seg - 1 + lf;
      gc = gc < n_cols ? gc : n_cols - 1;
      t = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const int n = fdiv(gc, fd_hw), pix = gc - n * HW;
      off = (unsigned)(((n * T + t) * HW + pix) * cs + half * 4) * 4u;
    } else if (I < G::NI) {
      const int s = (I - G::RAW_I) * 64 + lane;  // (e, co, stored half)
      const int e = s / (2 * G::CB), co = (s >> 1) % G::CB, half = (s & 1) ^ ((co >> 3) & 1);
      off = (unsigned)((e * CO + co0 + co) * 8 + half * 4) * 4u;
    }
    d_off[j] = off;
  }
  auto issue = [&](int k, int stage) __attribute__((always_inline)) {
    const char* xk = reinterpret_cast<const char*>(x + k * kstride);
    const char* uk = reinterpret_cast<const char*>(U + (size_t)k * 6 * CO * 8);
#pragma unroll
    for (int j = 0; j < DMAX; ++j) {
      if (j == DMIN && !more) break;  // wave-uniform
      const int I = wid + 4 * j;
      if constexpr ((EPI & 4096) != 0) if (I >= G::RAW_I) continue;  // knock-out: no U DMAs
      if constexpr ((EPI & 8192) != 0) if (I < G::RAW_I) continue;   // knock-out: no raw DMAs
      const char* src = (I < G::RAW_I ? xk : uk) + d_off[j];
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + stage * G::STAGE + I * 1024), 16,
                                       0, 0);
    }
  };
  // the lane's reads: raw frames of its tile column (m-tiles 2w, 2w+1 share a column group and are
  // adjacent in time), U fragments (co = 16 nt + l16, channel pair q)
  constexpr bool COLS = TS == 1;  // the wave's 2 tiles side by side (column groups), not in time
  const int j0 = 2 * wid;
  const int c_rd = (j0 / TS) * 16 + l16;
  const int rd_off = (4 * (j0 % TS)) * (G::P * 8) + (c_rd * 2 + ((q >> 1) ^ ((c_rd >> 3) & 1))) * 4 + (q & 1) * 2;
  const int c_rd1 = c_rd + 16;  // COLS: the second tile's column
  const int rd_off1 = (c_rd1 * 2 + ((q >> 1) ^ ((c_rd1 >> 3) & 1))) * 4 + (q & 1) * 2;
  const int u_rd = G::RAW_I * 256 + (l16 * 2 + ((q >> 1) ^ ((l16 >> 3) & 1))) * 4 + (q & 1) * 2;  // floats
  const int t0w = t_seg + 4 * (j0 % TS);
  const bool pad_lo = t0w == 0, pad_hi = t0w + (COLS ? 4 : 8) >= T;

  f32x4 acc[6][2][NT];
#pragma unroll
  for (int e = 0; e < 6; ++e)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[e][m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(k0, 0);
  __builtin_amdgcn_sched_barrier(0);
  for (int k = k0; k < k1; ++k) {
    // (EPI >= 256: convbench timing knock-outs, results wrong: 256 no transform VALU, 512 no DMAs in
    // the loop, 1024 no epilogue, 2048 no wait / barrier, 4096 no U DMAs, 8192 no raw DMAs)
    if constexpr ((EPI & 2048) == 0) {
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): chunk k's DMAs (own) landed
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();        // everyone's landed; everyone done with the other stage
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((EPI & 512) == 0)
      if (k + 1 < k1) issue(k + 1, (k + 1 - k0) & 1);
    __builtin_amdgcn_sched_barrier(0);
    const float* st = reinterpret_cast<const float*>(smem + ((k - k0) & 1) * G::STAGE);
    // frames of tile m: d[4m .. 4m + 5] (in time), or d[6m .. 6m + 5] (COLS: the m-th column group)
    constexpr int ND = COLS ? 12 : 10, MS = COLS ? 6 : 4;
    f32x2 d[ND];
#pragma unroll
    for (int f = 0; f < ND; ++f)
      d[f] = *reinterpret_cast<const f32x2*>(st + (COLS && f >= 6 ? rd_off1 + (f - 6) * (G::P * 8) : rd_off + f * (G::P * 8)));
    if (pad_lo) {
      d[0] = f32x2{0.f, 0.f};
      if constexpr (COLS) d[6] = f32x2{0.f, 0.f};
    }
    if (pad_hi) {
      d[ND - 1] = f32x2{0.f, 0.f};
      if constexpr (COLS) d[5] = f32x2{0.f, 0.f};
    }
    // B^T row e of tile m, formed right before its MFMAs (the 12 transformed values of both tiles
    // held at once, beside the 192-register accumulator, spilled at NT = 4); the same expressions
    // as the reference kernel, per element
    auto vrow = [&](int m, int e) __attribute__((always_inline)) {
      f32x2 r;
      if constexpr ((EPI & 256) != 0) {
        r = d[MS * m + e];
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const float d0 = d[MS * m][s2], d1 = d[MS * m + 1][s2], d2 = d[MS * m + 2][s2], d3 = d[MS * m + 3][s2],
                      d4 = d[MS * m + 4][s2], d5 = d[MS * m + 5][s2];
          float x;
          if (e == 0) x = 4.f * d0 - 5.f * d2 + d4;
          else if (e == 1) { const float e1 = d3 + d4, e2 = d1 + d2; x = e1 - 4.f * e2; }
          else if (e == 2) { const float e3 = d4 - d3, e4 = d1 - d2; x = e3 + 4.f * e4; }
          else if (e == 3) x = (d4 - d2) + 2.f * (d3 - d1);
          else if (e == 4) x = (d4 - d2) - 2.f * (d3 - d1);
          else x = 4.f * d1 - 5.f * d3 + d5;
          r[s2] = x;
        }
      }
      return r;
    };
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      f32x2 v[2][6];
      v[0][e] = vrow(0, e);
      v[1][e] = vrow(1, e);
      f32x2 u[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) u[nt] = *reinterpret_cast<const f32x2*>(st + u_rd + (e * G::CB + nt * 16) * 8);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[e][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[nt][s2], v[m][e][s2], acc[e][m][nt], 0, 0, 0);
    }
  }

  if constexpr ((EPI & 1024) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 6; ++e)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) sum += acc[e][m][nt][0] + acc[e][m][nt][1] + acc[e][m][nt][2] + acc[e][m][nt][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  // epilogue: y = A^T M in registers, 16-B bias / residual loads and stores
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = SPLIT ? p.part + (size_t)split * ((size_t)p.N * T * HW * CO) : reinterpret_cast<float*>(p.y);
  const size_t fstride = (size_t)HW * CO;
  // every N tile's bias before the first store, then one explicit vmcnt(0): a bias load issued after a
  // store waits for it (vmcnt retires in order; the compiler's waits in the per-tile branches were
  // vmcnt(0)), so the per-tile form paid the store latency once per (m, N tile)
  f32x4 bvs[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    bvs[nt] = (p.bias && !SPLIT) ? *reinterpret_cast<const f32x4*>(p.bias + co0 + 16 * nt + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int gc = col0 + c_rd + (COLS ? 16 * m : 0);
    const bool ok = gc < n_cols;
    const int gcc = ok ? gc : 0;
    const int n = fdiv(gcc, fd_hw), pix = gcc - n * HW;
    const int t0 = t0w + (COLS ? 0 : 4 * m);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = co0 + 16 * nt + 4 * q;
      const size_t o = ((size_t)(n * T + t0) * HW + pix) * CO + co;
      const f32x4 bv = bvs[nt];
      f32x4 rv[4];
#pragma unroll
      for (int a2 = 0; a2 < 4; ++a2)
        rv[a2] = ((EPI & 1) && ok) ? *reinterpret_cast<const f32x4*>(res + o + a2 * fstride) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 m0 = acc[0][m][nt], m1 = acc[1][m][nt], m2 = acc[2][m][nt], m3 = acc[3][m][nt],
                  m4 = acc[4][m][nt], m5 = acc[5][m][nt];
      const f32x4 s12 = m1 + m2, d12 = psub4(m1, m2), s34 = m3 + m4, d34 = psub4(m3, m4);
      f32x4 yv[4];
      yv[0] = m0 + s12 + s34;
      yv[1] = d12 + 2.f * d34;
      yv[2] = s12 + 4.f * s34;
      yv[3] = d12 + 8.f * d34 + m5;
      if (ok) {
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) {
          f32x4 vv = SPLIT ? yv[a2] : yv[a2] + bv;
          if constexpr (EPI & 1) vv += rv[a2];
          if constexpr (EPI & 2) {
#pragma unroll
            for (int c = 0; c < 4; ++c) vv[c] = relu1(vv[c]);
          }
          if constexpr ((EPI & 32768) != 0)
            __builtin_nontemporal_store(vv, reinterpret_cast<f32x4*>(yout + o + a2 * fstride));
          else
            *reinterpret_cast<f32x4*>(yout + o + a2 * fstride) = vv;
        }
      }
    }
  }
}

template <int TS, int NT, int EPI>
hipError_t winot5_launch_e(const ConvParams& p, hipStream_t s) {
  using G = T5<TS, NT>;
  static bool attr = false;
  if (!attr && G::LDS > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_winot5<TS, NT, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int n_cols = p.N * p.Hi * p.Wi;
  const int n_seg = (p.Ti / 4) / TS;
  const int n_co = p.Cout / G::CB;
  const int nb = ((n_cols + G::P - 1) / G::P) * n_seg * n_co * ((EPI & 4) ? p.n_split : 1);
  hipLaunchKernelGGL((conv_winot5<TS, NT, EPI>), dim3(nb), dim3(256), G::LDS, s, p, n_co, n_seg, n_cols,
                     fast_div(p.Hi * p.Wi));
  return hipGetLastError();
}

// W3 (NT = 2 only): three waves per SIMD (EPI bit 16384: 160 VGPRs, three 48 KiB blocks per CU)
template <int TS, int NT, bool W3 = false>
hipError_t winot5_launch(const ConvParams& p, hipStream_t s) {
  constexpr int X = W3 ? 16384 : 0;
  if (p.n_split > 1) {
    hipError_t e = winot5_launch_e<TS, NT, 4 + X>(p, s);  // bias, residual and ReLU in the sum pass
    if (e != hipSuccess) return e;
    return launch_split_sum(p, s);
  }
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 2: return winot5_launch_e<TS, NT, 2 + X>(p, s);  // TP1 / stem T: BN + ReLU
    case 3: return winot5_launch_e<TS, NT, 3 + X>(p, s);  // TP2: BN + residual + ReLU
    case 1: return winot5_launch_e<TS, NT, 1 + X>(p, s);
    default: return winot5_launch_e<TS, NT, 0 + X>(p, s);
  }
}

// Channels per wave: 64 (NT = 4, two blocks per CU: 512 slots) or 32 (NT = 2 at three waves per SIMD,
// three blocks per CU: 768 slots), whichever fills its last wave of blocks better, NT = 2 priced at
// its measured 5.4 % more time per output on a full chip (profiles/r05v_winot_nt2_three_waves.txt:
// 0.832 vs 0.789 ms). Layer3 at 30 clips: 736 NT-4 blocks fill 1.44 waves (0.72), 1472 NT-2 blocks
// 1.92 (0.96 / 1.054 = 0.91). Both forms compute the same products in the same order
// (bit-identical), so the batch-dependent choice does not change a clip's result. Returns 4, 2 or 3
// (NT = 2 at three waves per SIMD); *blocks: the launch's blocks.
int winot5_nt(const ConvParams& p, long* blocks) {
  const int tt = p.Ti / 4;
  const int ts = tt % 4 == 0 ? 4 : tt % 2 == 0 ? 2 : 1;
  const long b4 = (long)((p.N * p.Hi * p.Wi + 16 * 8 / ts - 1) / (16 * 8 / ts)) * (tt / ts) * (p.Cout / 64);
  const long b2 = 2 * b4;
  const double fill4 = (double)b4 / (double)(((b4 + 511) / 512) * 512);
  const double fill2 = (double)b2 / (double)(((b2 + 767) / 768) * 768) / 1.054;
  // (TS = 1: three 60 KiB NT-2 blocks do not fit a CU's LDS; the two-wave NT-2 form below 512 blocks)
  const int nt = ts == 1 ? (b4 >= 512 ? 4 : 2) : fill2 > fill4 ? 3 : 4;
  if (blocks) *blocks = nt == 4 ? b4 : b2;
  return nt;  // (ts == 1 never returns 3)
}

// force_nt (tools/convbench): 4, 2 (NT = 2 at two waves per SIMD) or 3 (NT = 2 at three)
hipError_t winot5_dispatch(const ConvParams& p, hipStream_t s, int force_nt = 0) {
  const int tt = p.Ti / 4;
  const int ts = tt % 4 == 0 ? 4 : tt % 2 == 0 ? 2 : 1;
  const int nt = force_nt ? force_nt : winot5_nt(p, nullptr);
  if (ts == 4) return nt == 4 ? winot5_launch<4, 4>(p, s) : nt == 3 ? winot5_launch<4, 2, true>(p, s) : winot5_launch<4, 2>(p, s);
  if (ts == 1) return nt == 4 ? winot5_launch<1, 4>(p, s) : nt == 3 ? winot5_launch<1, 2, true>(p, s) : winot5_launch<1, 2>(p, s);
  return nt == 4 ? winot5_launch<2, 4>(p, s) : nt == 3 ? winot5_launch<2, 2, true>(p, s) : winot5_launch<2, 2>(p, s);
}

// conv_winot5 addresses its input with 32-bit byte offsets from the chunk's scalar base
bool winot5_fits(const ConvParams& p) { return (size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin * 4 < ((size_t)1 << 32); }

}  // namespace

bool winot_c8_ok(const ConvParams& p) {
  return winot_supported(p) && !(p.vflags & CLASFV_VARIANT_WINOT_REFERENCE) && p.Ti % 8 == 0 && winot5_fits(p);
}

// conv_winot5 for channels-last input: T % 8 == 0 in time-adjacent tile pairs, other T % 4 == 0 (one
// tile row per segment) in column-adjacent pairs (TS = 1); CLASFV_VARIANT_WINOT_NO_TS1 keeps the
// latter on conv_winot
static bool winot5_ok(const ConvParams& p) {
  if (winot_c8_ok(p)) return true;
  return !(p.vflags & (CLASFV_VARIANT_WINOT_NO_TS1 | CLASFV_VARIANT_WINOT_REFERENCE)) && !p.x_c8 && winot_supported(p) &&
         winot5_fits(p);
}

// Split-K factor for conv_winot5 (ConvParams::n_split). Layer4 at 112x112 clips (4 x 7 x 7 output
// voxels per clip) runs 192 blocks for 30 clips: one per CU on three quarters of the chip, one wave per
// SIMD. Maps of <= 256 output voxels per clip split their input channels into 4 ranges of >= 8 chunks
// (768 blocks for 30 clips). The factor depends on the per-clip shape only, never on the batch size,
// so a clip's result does not depend on the clips batched with it.
int winot_split_for(const ConvParams& p) {
  if (!winot5_ok(p) || p.x_c8 || (p.vflags & CLASFV_VARIANT_NO_SPLIT_K)) return 1;
  if ((long)p.To * p.Ho * p.Wo > 256 || p.Cin / 8 < 4 * 8) return 1;
  return 4;
}

bool winot_supported(const ConvParams& p) {
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && p.KT == 3 && p.KH == 1 && p.KW == 1 && p.st == 1 &&
         p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 0 && p.pw == 0 && p.Cin % 8 == 0 && p.Cout % BN == 0 &&
         p.To == p.Ti && p.Ti % 4 == 0 && p.Ho == p.Hi && p.Wo == p.Wi &&
         (size_t)p.N * p.Ti * p.Hi * p.Wi * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31);
}

// U: [Cin/8][6][Cout/64][64][8] transformed weights (winot_transform_weights).
hipError_t launch_winot(const ConvParams& p, hipStream_t s) {
  if (!winot_supported(p)) return hipErrorInvalidValue;
  // CLASFV_VARIANT_WINOT_REFERENCE (tests): always conv_winot; both kernels compute the same products in
  // the same order (bit-identical outputs).
  if (winot5_ok(p)) return winot5_dispatch(p, s);
  if (p.x_c8) return hipErrorInvalidValue;  // 8-channel-blocked input: conv_winot5 only
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
// tools/convbench.hip: run one temporal kernel variant (0 conv_winot, 500 conv_winot5); timing and
// bit-identity comparisons only, not product code.
hipError_t launch_winot_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (p.x_c8 && ko == 0) return hipErrorInvalidValue;
  switch (ko) {
    case 0: {
      hipError_t e = hipFuncSetAttribute((const void*)conv_winot, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      if (e != hipSuccess) return e;
      const int n_tiles = p.N * (p.Ti / 4) * p.Hi * p.Wi;
      hipLaunchKernelGGL(conv_winot, dim3(((n_tiles + BT - 1) / BT) * (p.Cout / BN)), dim3(NTHR), LDS_BYTES, s, p,
                         p.Cout / BN, n_tiles);
      return hipGetLastError();
    }
    case 500: return p.x_c8 && !winot_c8_ok(p) ? hipErrorInvalidValue : winot5_dispatch(p, s);
    // knock-outs (TS = 4, NT = 4, EPI 2 + bits): 801 no transform, 802 no loop DMAs, 804 no epilogue,
    // 808 no wait / barrier, 815 all
    case 801: return winot5_launch_e<4, 4, 2 + 256>(p, s);
    case 802: return winot5_launch_e<4, 4, 2 + 512>(p, s);
    case 804: return winot5_launch_e<4, 4, 2 + 1024>(p, s);
    case 808: return winot5_launch_e<4, 4, 2 + 2048>(p, s);
    case 815: return winot5_launch_e<4, 4, 2 + 256 + 512 + 1024 + 2048>(p, s);
    case 816: return winot5_launch_e<4, 4, 2 + 4096>(p, s);   // no U DMAs in the loop
    case 832: return winot5_launch_e<4, 4, 2 + 8192>(p, s);   // no raw DMAs in the loop
    case 817: return winot5_launch_e<4, 4, 3 + 4096>(p, s);   // (residual form)
    case 833: return winot5_launch_e<4, 4, 3 + 8192>(p, s);
    case 502: return winot5_dispatch(p, s, 2);
    case 503: return winot5_dispatch(p, s, 3);  // NT 2, three waves per SIMD
    case 504: return winot5_dispatch(p, s, 4);
  }
  if (ko >= 600 && ko < 700 && p.part && !p.x_c8) {  // split-K: 6 NT S (p.part holds 8 partials)
    ConvParams q = p;
    q.n_split = ko % 10;
    return q.n_split > 8 ? hipErrorInvalidValue : winot5_dispatch(q, s, (ko / 10) % 10);
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
