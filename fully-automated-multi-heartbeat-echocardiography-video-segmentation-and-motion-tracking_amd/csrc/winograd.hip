// Fused Winograd F(2x2, 3x3) convolution for the stride-1 1x3x3 spatial convs of R(2+1)D-18 (fp32).
//
// Reference op: the Conv2Plus1D spatial conv3d(kernel (1,3,3), stride 1, padding (0,1,1)) + BN(eval)
// + ReLU of torchvision's r2plus1d_18 (called from src/model/R2plus1D_18_MotionNet.py:29-37). On
// NVIDIA this is what cuDNN's Winograd algorithms compute; here it is one hand-written kernel.
//
//   Y(2x2 tile) = A^T [ sum_ci U_ci (.) V_ci ] A,   U = G g G^T (host, double),  V = B^T d B
//
// so 16 multiplies per 2x2 outputs and input channel instead of 36: the 16 transform elements
// e = 4i + j become 16 independent GEMMs M_e[tile][co] = sum_ci V_e[tile][ci] U_e[ci][co], run on
// exact-fp32 v_mfma_f32_16x16x4_f32.
//
// Block = 32 output tiles (2x2 pixels each, flattened over N,T,H/2,W/2) x 16*NT output channels,
// 4 waves; wave w owns the transform row i = w (e = 4w..4w+3). Per chunk of 8 input channels:
//  * raw 4x4 input patches (32 tiles x 16 pixels x 32 B = 16 KB) arrive by LDS-DMA
//    (global_load_lds_dwordx4) into a 2-deep ring; pixel slot px of tile t is stored at
//    px ^ (t & 7), which makes the transform's ds_read_b32 conflict-free;
//  * all 256 threads transform one (tile, channel) patch each into V (16 KB, double-buffered,
//    layout [e][tile][8 ci]) -- the next chunk's transform overlaps this chunk's MFMAs;
//  * U_e for the wave's 4 e's comes straight from global memory (16-B loads, [chunk][i][co][8 ci][j]),
//    prefetched two chunks ahead into registers;
//  * 2 K steps x 4 e x 2 m tiles x NT MFMAs per chunk and wave, one barrier per chunk.
// Epilogue: each wave applies the column half of the inverse transform to its row of M in registers,
// the row half goes through LDS (one barrier), then bias, residual and ReLU on the 2x2 output pixels.
#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BT = 32;                 // tiles per block
constexpr int RAW_BYTES = BT * 16 * 32;  // 16 KB: [tile][px'][8 ci]
constexpr int V_BYTES = 16 * BT * 32;    // 16 KB: [e][tile][8 ci]
constexpr int RAW_STAGES = 3;            // raw ring depth: chunk k+3 is fetched while k+1 is transformed

__device__ inline int xcd_swizzle_w(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// NCH > 0: the chunk count Cin/8 as a compile-time constant -> the chunk loop is fully unrolled and
// the compiler's own vmcnt waits are exact (the runtime loop makes it wait for the previous chunk's
// fetches too, one chunk early).
template <int NT, int NCH = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wino(ConvParams p, int n_co,
                                                                                             int n_tiles, FastDiv fd_f,
                                                                                             FastDiv fd_x) {
  __shared__ __align__(16) char smem[RAW_STAGES * RAW_BYTES + 2 * V_BYTES];
  char* raw = smem;
  char* vbuf = smem + RAW_STAGES * RAW_BYTES;

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_w(blockIdx.x, gridDim.x);
  // Block order (one XCD runs a contiguous range of it): groups of G co blocks outermost, then tile
  // blocks, then the G co blocks of the group -- an XCD's co-resident blocks then need the U slices of
  // G co blocks (<= 3 MB at layer3/4 widths, L2-resident) instead of all n_co (9.4 / 38 MB, which
  // every tile block re-streamed from the fabric: FETCH 27x the algorithmic bytes).
  const int G = n_co % 4 == 0 ? 4 : n_co % 3 == 0 ? 3 : n_co % 2 == 0 ? 2 : 1;
  const int n_tb = (n_tiles + BT - 1) / BT;
  const int grp = blk / (n_tb * G), grem = blk - grp * (n_tb * G);
  const int t0 = (grem / G) * BT, n0 = (grp * G + grem % G) * 16 * NT;
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int TY = (H + 1) >> 1, TX = (W + 1) >> 1;
  const int nchunk = NCH > 0 ? NCH : C >> 3;

  // ---- per-lane DMA sources: instruction j of this wave fills 16-B slot s = (wid + 4j)*64 + lane
  int d_off[4];  // float offset of channel 0 of the source pixel, or -1 (zero padding)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int s = (wid + 4 * j) * 64 + lane;
    const int tl = s >> 5, px = ((s & 31) >> 1) ^ (tl & 7), half = s & 1;
    const int tg = t0 + tl;
    int off = -1;
    if (tg < n_tiles) {
      const int f = fdiv(tg, fd_f), r = tg - f * (TY * TX);
      const int ty = fdiv(r, fd_x), tx = r - ty * TX;
      const int yy = 2 * ty - 1 + (px >> 2), xx = 2 * tx - 1 + (px & 3);
      if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = ((f * H + yy) * W + xx) * C + half * 4;
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int chunk, int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const void* src = (d_off[j] >= 0 && chunk >= 0) ? (const void*)(x + (size_t)d_off[j] + chunk * 8) : p.zero;
      char* dst = raw + buf * RAW_BYTES + (wid + 4 * j) * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  // ---- transform: thread = (tile tt, channel cc) of the chunk
  const int tt = tid >> 3, cc = tid & 7;
  // The transform is split so that the raw reads of chunk k+1 are issued before the MFMAs of chunk
  // k and its arithmetic + V stores fill their issue gaps (sched_group_barrier in step()).
  auto transform_read = [&](int buf_raw, float (&d)[16]) {
    const float* rb = reinterpret_cast<const float*>(raw + buf_raw * RAW_BYTES) + tt * 128 + cc;
#pragma unroll
    for (int px = 0; px < 16; ++px) d[px] = rb[(px ^ (tt & 7)) * 8];
  };
  auto transform_write = [&](const float (&d)[16], int buf_v) {
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // B^T d
      t[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
      t[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
      t[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
      t[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
    // V[e][tile & 15][(ci >> 1) ^ sw][tile >> 4][ci & 1], sw = ((tile & 15) >> 2) & 2: one lane's A
    // operands of both m tiles and both K steps are 16 contiguous bytes, and the swizzle puts every
    // 16-lane group of the ds_read_b128 on distinct bank quads (see conv_wino_q)
    float* vb = reinterpret_cast<float*>(vbuf + buf_v * V_BYTES) +
                (((tt & 15) * 4 + ((cc >> 1) ^ (((tt & 15) >> 2) & 2))) * 2 + (tt >> 4)) * 2 + (cc & 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // (B^T d) B
      vb[(4 * r + 0) * BT * 8] = t[4 * r + 0] - t[4 * r + 2];
      vb[(4 * r + 1) * BT * 8] = t[4 * r + 1] + t[4 * r + 2];
      vb[(4 * r + 2) * BT * 8] = t[4 * r + 2] - t[4 * r + 1];
      vb[(4 * r + 3) * BT * 8] = t[4 * r + 1] - t[4 * r + 3];
    }
  };

  // ---- U operands: lane (co = l16, q) of wave (e row) i, n tile nt reads the 8 floats
  // U[chunk][i][co][q][j][s] (e = 4i + j, ci = 8 chunk + 2q + s) as two 16-B loads.
  const float* ub = U + (((size_t)wid * CO + n0 + l16) * 4 + q) * 8;
  f32x4 u0[NT][2], u1[NT][2], u2[NT][2];
  auto load_u = [&](int chunk, f32x4 (&u)[NT][2]) {
    const float* b = ub + (size_t)chunk * 4 * CO * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int h = 0; h < 2; ++h) u[nt][h] = *reinterpret_cast<const f32x4*>(b + (size_t)nt * 16 * 32 + h * 4);
  };
  // Every fetch is issued unconditionally (past-the-end chunks re-read chunk 0 / the zero block into
  // slots nobody reads again), so the number of memory operations per chunk is a constant and the
  // waits below are exact: vmcnt(16) = "everything but the previous chunk's 4 DMAs + 12 U loads".
  static_assert(4 + 2 * NT == 10, "wait counts assume NT = 3");
  f32x4 acc[4][2][NT];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[j][m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: raw(0..2), U(0..1); transform(0)
  // (the sched_barriers pin the issue order the counted vmcnt below relies on)
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  load_u(0, u0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(nchunk > 1 ? 1 : -1, 1);
  __builtin_amdgcn_sched_barrier(0);
  load_u(nchunk > 1 ? 1 : 0, u1);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(nchunk > 2 ? 2 : -1, 2);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | (20 & 15) | ((20 >> 4) << 14));  // vmcnt(20): raw(0) landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  {
    float d[16];
    transform_read(0, d);
    transform_write(d, 0);
  }

  const int a_off = (l16 * 4 + (q ^ ((l16 >> 2) & 2))) * 16;  // the lane's 4 V values inside one e slice
  // One chunk k: U(k) is in `uc`, U(k+2) is fetched into `un` (3-way rotation, no register copies);
  // raw(k+3) is fetched into the ring slot raw(k) used; raw(k+1) is transformed into V[(k+1)&1]
  // while the MFMAs consume V[k&1].
  auto step = [&](int k, f32x4 (&uc)[NT][2], f32x4 (&un)[NT][2]) {
    // raw(k+1) and U(k) were issued two chunks ago; only chunk k-1's 10 fetches may be in flight.
    __builtin_amdgcn_s_waitcnt(0x0070 | 10);  // vmcnt(10) lgkmcnt(0): own V stores done before the barrier
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue_raw(k + 3 < nchunk ? k + 3 : -1, k % RAW_STAGES);
    load_u(k + 2 < nchunk ? k + 2 : 0, un);
    __builtin_amdgcn_sched_barrier(0);
    const char* vb = vbuf + (k & 1) * V_BYTES + a_off;
    f32x4 a[4];  // {m0 s0, m0 s1, m1 s0, m1 s1} per j
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const f32x4*>(vb + (4 * wid + j) * (BT * 32));
    // transform raw(k+1) -> V[(k+1)&1] (on the last chunk it transforms the ring's past-the-end
    // fetch into the V buffer nobody reads again: branch-free keeps one scheduling region)
    float d[16];
    transform_read((k + 1) % RAW_STAGES, d);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            acc[j][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][2 * m + s], uc[nt][j >> 1][(j & 1) * 2 + s],
                                                                 acc[j][m][nt], 0, 0, 0);
          }
    transform_write(d, (k + 1) & 1);
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
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  };
  if constexpr (NCH > 0) {
#pragma unroll
    for (int kk = 0; kk < NCH; kk += 3) {
      step(kk, u0, u2);
      if (kk + 1 < NCH) step(kk + 1, u1, u0);
      if (kk + 2 < NCH) step(kk + 2, u2, u1);
    }
  } else {
    // Full triples branch-free, then the tail.
    int k = 0;
    for (; k + 3 <= nchunk; k += 3) {
      step(k, u0, u2);
      step(k + 1, u1, u0);
      step(k + 2, u2, u1);
    }
    if (k < nchunk) step(k, u0, u2);
    if (k + 1 < nchunk) step(k + 1, u1, u0);
  }

  // ---- epilogue: Y = A^T M A. Wave i holds row i of M: the column combination (. A) is done in
  // registers, Z_i = (M_i0 + M_i1 + M_i2, M_i1 - M_i2 - M_i3); the row combination (A^T .) needs all
  // four waves and goes through LDS: Z[i][tile][co][2] (48 KB), one barrier.
  // Unit = (tile, 4 consecutive channels): 16-B bias / residual loads and 16-B stores. All of a
  // thread's global loads are issued before the LDS exchange (their latency hides behind it, and
  // res may alias y: no load can then wait behind a store).
  constexpr int CQ = 4 * NT, UNITS = BT * CQ, UPT = (UNITS + 255) / 256;
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  size_t u_o[UPT];
  int u_ok[UPT], u_z[UPT];
  f32x4 u_b[UPT], u_r[UPT][4];
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    const int un = tid + 256 * u;
    const int tl = un / CQ, cq = un - tl * CQ;
    const int tg = t0 + tl;
    const bool live = un < UNITS && tg < n_tiles;
    const int tgc = live ? tg : t0;
    const int f = fdiv(tgc, fd_f), rem = tgc - f * (TY * TX);
    const int ty = fdiv(rem, fd_x), tx = rem - ty * TX;
    const int co = n0 + 4 * cq;
    u_o[u] = ((size_t)(f * H + 2 * ty) * W + 2 * tx) * CO + co;
    u_z[u] = tl * (16 * NT) + 4 * cq;
    int ok = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        if (live && 2 * ty + a < H && 2 * tx + b < W) ok |= 1 << (2 * a + b);
    u_ok[u] = ok;
    u_b[u] = (p.bias && live) ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int px = 0; px < 4; ++px)
      u_r[u][px] = (res && (ok >> px & 1))
                       ? *reinterpret_cast<const f32x4*>(res + u_o[u] + (size_t)((px >> 1) * W + (px & 1)) * CO)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x2* zs = reinterpret_cast<f32x2*>(smem);
  __syncthreads();  // everyone is done with raw / V
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float m0 = acc[0][m][nt][r], m1 = acc[1][m][nt][r], m2 = acc[2][m][nt][r], m3 = acc[3][m][nt][r];
        zs[(wid * BT + m * 16 + 4 * q + r) * (16 * NT) + nt * 16 + l16] = f32x2{m0 + m1 + m2, m1 - m2 - m3};
      }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    if (!u_ok[u]) continue;
    // z[i][h]: channels 2h, 2h+1 of row i as {c.col0, c.col1, c'.col0, c'.col1}
    f32x4 z[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4* zp = reinterpret_cast<const f32x4*>(zs + i * BT * (16 * NT) + u_z[u]);
      z[i][0] = zp[0];
      z[i][1] = zp[1];
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int px = 2 * a + b;
        if (!(u_ok[u] >> px & 1)) continue;
        f32x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int h = c >> 1, e = (c & 1) * 2 + b;
          const float y = a == 0 ? z[0][h][e] + z[1][h][e] + z[2][h][e] : z[1][h][e] - z[2][h][e] - z[3][h][e];
          float o = y + u_b[u][c];
          if (res) o += u_r[u][px][c];
          if (p.relu) o = relu1(o);
          v[c] = o;
        }
        *reinterpret_cast<f32x4*>(yout + u_o[u] + (size_t)(a * W + b) * CO) = v;
      }
  }
}

}  // namespace

bool wino_supported(const ConvParams& p) {
  return !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && p.KT == 1 && p.KH == 3 && p.KW == 3 && p.sh == 1 &&
         p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Cin % 16 == 0 && p.Cout % 48 == 0 &&
         p.Ho == p.Hi && p.Wo == p.Wi && p.To == p.Ti &&
         (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31);
}

// U: [Cin/8][4][Cout][4][4][2] transformed weights (wino_transform_weights).
hipError_t launch_wino(const ConvParams& p, hipStream_t s) {
  if (!wino_supported(p)) return hipErrorInvalidValue;
  const int n_tiles = p.N * p.To * ((p.Ho + 1) / 2) * ((p.Wo + 1) / 2);
  const int n_co = p.Cout / 48;
  const int nb = (n_tiles + BT - 1) / BT;
  const int tx = (p.Wo + 1) / 2, ty = (p.Ho + 1) / 2;
  const FastDiv fd_f = fast_div(tx * ty), fd_x = fast_div(tx);
  switch (p.Cin >> 3) {  // fully unrolled chunk loops for the layer1..4 widths
    case 8: hipLaunchKernelGGL((conv_wino<3, 8>), dim3(nb * n_co), dim3(256), 0, s, p, n_co, n_tiles, fd_f, fd_x); break;
    case 16: hipLaunchKernelGGL((conv_wino<3, 16>), dim3(nb * n_co), dim3(256), 0, s, p, n_co, n_tiles, fd_f, fd_x); break;
    case 32: hipLaunchKernelGGL((conv_wino<3, 32>), dim3(nb * n_co), dim3(256), 0, s, p, n_co, n_tiles, fd_f, fd_x); break;
    case 64: hipLaunchKernelGGL((conv_wino<3, 64>), dim3(nb * n_co), dim3(256), 0, s, p, n_co, n_tiles, fd_f, fd_x); break;
    default: hipLaunchKernelGGL((conv_wino<3, 0>), dim3(nb * n_co), dim3(256), 0, s, p, n_co, n_tiles, fd_f, fd_x); break;
  }
  return hipGetLastError();
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: 0 = product dispatch, 100 = the runtime-chunk-loop instance
hipError_t launch_wino_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (ko != 100) return launch_wino(p, s);
  const int n_tiles = p.N * p.To * ((p.Ho + 1) / 2) * ((p.Wo + 1) / 2);
  const int n_co = p.Cout / 48;
  const int tx = (p.Wo + 1) / 2, ty = (p.Ho + 1) / 2;
  hipLaunchKernelGGL((conv_wino<3, 0>), dim3(((n_tiles + BT - 1) / BT) * n_co), dim3(256), 0, s, p, n_co, n_tiles,
                     fast_div(tx * ty), fast_div(tx));
  return hipGetLastError();
}
#endif

// Host: U[c/8][i][o][(c%8)/2][j][c%2] = (G g_{o,c} G^T)[i][j] in double, g = folded 3x3 kernel.
void wino_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  for (size_t i = 0; i < (size_t)16 * cin_p * cout_p; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* g = w + ((size_t)o * cin + c) * 9;
      double tmp[4][3];
      for (int i = 0; i < 4; ++i)
        for (int v = 0; v < 3; ++v) tmp[i][v] = G[i][0] * g[0 * 3 + v] + G[i][1] * g[1 * 3 + v] + G[i][2] * g[2 * 3 + v];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          const double u = tmp[i][0] * G[j][0] + tmp[i][1] * G[j][1] + tmp[i][2] * G[j][2];
          U[((((size_t)(c / 8) * 4 + i) * cout_p + o) * 4 + (c % 8) / 2) * 8 + j * 2 + (c % 2)] = (float)u;
        }
    }
}
