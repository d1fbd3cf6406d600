// Patch-tiled fused Winograd F(2x4, 3x3) for the widest stride-1 1x3x3 fp32 convs (R(2+1)D-18
// layer1 at 32x112x112 clips: 56x56 maps; layer1+2 at 224x224). Same op as conv_wino_q
// (winograd2.hip) -- the Conv2Plus1D spatial conv3d(kernel (1,3,3), padding (0,1,1)) + BN(eval)
// (+ residual) + ReLU of torchvision's r2plus1d_18, called from src/model/R2plus1D_18_MotionNet.py:29-37
// -- with a larger output tile: 2 rows x 4 columns, F(2,3) along H and F(4,3) along W,
//
//   Y(2x4) = A2^T [ sum_ci U_ci (.) V_ci ] A4,   U = G2 g G4^T (host, double),  V = B2^T d B4
//
// 24 multiplies per 8 outputs and input channel (3 per output) instead of F(2x2)'s 16 per 4 (4 per
// output): 25 % fewer MFMAs. The F(4,3) factors are those of the temporal kernel (winograd_t.hip).
//
// Block = 4 waves (wave = H-transform row i, owning e = 6i .. 6i+5) x 16 tiles (2 patches of 4x2
// tiles = 8x8 output pixels, the 10x10-pixel input patches of conv_wino_q) x 48 output channels, 2
// blocks per CU (60 KB LDS). Per chunk of 8 input channels:
//  * raw patches by LDS-DMA (2 instructions per wave) into a ring of 3. The patch image is remapped
//    (pixel column c at c + c/4, patch 1 at +122 pixels) so that the transform's ds_read_b32 lane
//    groups -- 2 patches x 2 tile columns x 8 channels -- hit 32 distinct banks;
//  * the transform of chunk k+2 (thread = (W half jh, tile, channel): 20 raw values -> 12 of the 24
//    V values) is split around chunk k's MFMAs; V ring of 3, each chunk's A operands read into
//    registers one chunk ahead; U operands from global memory one chunk ahead (2-way rotation);
//  * 6 e x 2 K steps x 3 n tiles = 36 MFMAs per chunk and wave (conv_wino_q: 48).
// Epilogue: each wave applies A4^T to its row of M in registers; the four rows meet in LDS for A2^T,
// then bias, residual and ReLU, 16-B stores.
#include <type_traits>

#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ inline int xcd_swizzle_r(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ inline void dma16r(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

constexpr int R_BT = 16;                      // tiles per block
constexpr int R_RS = 12;                      // patch image row: 10 pixels at c + c/4 (pads at 4, 9)
constexpr int R_PP = 122;                     // patch 1 starts at pixel 122 (== 2 mod 4)
constexpr int R_RAW = 8 * 1024;               // 8 DMA wave-instructions = 256 pixel slots (244 used)
constexpr int R_V = 24 * R_BT * 32;           // 12 KB: [e][tile][8 ci]
constexpr int R_LDS = 3 * R_RAW + 3 * R_V;    // 60 KB
constexpr int R_Z = 4 * 4 * R_BT * 48 * 4;    // epilogue Z[i][b][tile][48 co]: 48 KB
static_assert(R_Z <= R_LDS, "epilogue exchange");

__device__ inline int rpos(int col) { return col + (col >> 2); }

template <int NCH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wino_r(ConvParams p, int n_co,
                                                                                             int n_patches) {
  __shared__ __align__(16) char smem[R_LDS];
  char* raw = smem;
  char* vbuf = smem + 3 * R_RAW;

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  const int blk = xcd_swizzle_r(blockIdx.x, gridDim.x);
  const int pg0 = (blk / n_co) * 2, n0 = (blk % n_co) * 48;
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int PY = H >> 3, PX = W >> 3;
  const int nchunk = NCH > 0 ? NCH : C >> 3;

  // raw DMA: instruction j of this wave fills slots s = (wid + 4j)*64 + lane = pixel s/2, half s&1
  int d_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int s = (wid + 4 * j) * 64 + lane;
    const int px = s >> 1, half = s & 1;
    const int pp = px >= R_PP ? 1 : 0, rem = px - pp * R_PP;
    const int row = rem / R_RS, pc = rem - row * R_RS;
    const int col = pc - (pc + 1) / 5;  // inverse of rpos (pads: pc == 4, 9)
    int off = -1;
    if (row < 10 && pc != 4 && pc != 9 && pg0 + pp < n_patches) {
      const int gp = pg0 + pp;
      const int f = gp / (PY * PX), r = gp - f * (PY * PX);
      const int pr = r / PX, pcx = r - pr * PX;
      const int yy = pr * 8 - 1 + row, xx = pcx * 8 - 1 + col;
      if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = ((f * H + yy) * W + xx) * C + half * 4;
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const void* src = (k < nchunk && d_off[j] >= 0) ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      dma16r(src, raw + stage * R_RAW + (wid + 4 * j) * 1024);
    }
  };
  // U: lane (co = l16, q) of wave (H row) i, n tile nt: 12 floats U[chunk][i][co][q][j][s]
  const float* ub = U + (((size_t)wid * CO + n0 + l16) * 4 + q) * 12;
  auto load_u = [&](int k, f32x4 (&u)[3][3]) __attribute__((always_inline)) {
    const float* b = ub + (size_t)(k < nchunk ? k : 0) * 4 * CO * 48;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int h = 0; h < 3; ++h) u[nt][h] = *reinterpret_cast<const f32x4*>(b + (size_t)nt * 16 * 48 + h * 4);
  };
  // transform thread: wave half jh = wid >> 1 (uniform), tile rows tr = 2*(wid & 1) + (lane >> 5),
  // patch pp = lane >> 4 & 1, tile column tc = lane >> 3 & 1, channel cc = lane & 7;
  // tile index = pp*8 + tr*2 + tc. It reads rows 0..3, columns jh..jh+4 of the tile's 4x6 window.
  const int jh = wid >> 1;
  const int t_tr = 2 * (wid & 1) + (lane >> 5), t_pp = (lane >> 4) & 1, t_tc = (lane >> 3) & 1, t_cc = lane & 7;
  const int t_tile = t_pp * 8 + t_tr * 2 + t_tc;
  const int raw_base = (t_pp * R_PP + 2 * t_tr * R_RS + 5 * t_tc) * 8 + t_cc;  // rpos(4 tc + c) = 5 tc + rpos(c)
  auto transform_read = [&](int rstage, float (&d)[4][5]) __attribute__((always_inline)) {
    const float* rb = reinterpret_cast<const float*>(raw + rstage * R_RAW) + raw_base;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c) d[r][c] = rb[(r * R_RS + rpos(jh + c)) * 8];
  };
  using JH0 = std::integral_constant<int, 0>;
  using JH1 = std::integral_constant<int, 1>;
  // JH = jh as a compile-time constant: the caller branches once per chunk loop on the wave-uniform
  // jh, so no branch splits a chunk's scheduling region
  auto transform_write = [&](auto jh_c, const float (&d)[4][5], int vstage) __attribute__((always_inline)) {
    constexpr int JH = decltype(jh_c)::value;
    // B2^T along H (rows), then B4^T along W for this thread's 3 of the 6 columns
    float t[4][5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      t[0][c] = d[0][c] - d[2][c];
      t[1][c] = d[1][c] + d[2][c];
      t[2][c] = d[2][c] - d[1][c];
      t[3][c] = d[1][c] - d[3][c];
    }
    float* vb = reinterpret_cast<float*>(vbuf + vstage * R_V) + t_tile * 8 + t_cc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float o[3];
      const float* T = t[i];
      if constexpr (JH == 0) {  // T[c] = D_c, c = 0..4
        o[0] = 4.f * T[0] - 5.f * T[2] + T[4];
        o[1] = (T[3] + T[4]) - 4.f * (T[1] + T[2]);
        o[2] = (T[4] - T[3]) + 4.f * (T[1] - T[2]);
      } else {  // T[c] = D_{c+1}, c = 0..4
        o[0] = (T[3] - T[1]) + 2.f * (T[2] - T[0]);
        o[1] = (T[3] - T[1]) - 2.f * (T[2] - T[0]);
        o[2] = 4.f * T[0] - 5.f * T[2] + T[4];
      }
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) vb[(i * 6 + 3 * JH + jj) * (R_BT * 8)] = o[jj];
    }
  };

  f32x4 uu[2][3][3];  // U operands, 2-way rotation (chunk k uses uu[k & 1])
  f32x2 aa[2][6];     // A operands (V of this wave's 6 e), 2-way rotation
  f32x4 acc[6][3];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) acc[j][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int a_off = (l16 * 8 + 2 * q) * 4;  // bytes: lane's (tile l16, ci 2q..2q+1) pair in an e slice
  auto read_a = [&](int vstage, f32x2 (&a)[6]) __attribute__((always_inline)) {
    const char* vb = vbuf + vstage * R_V + a_off;
#pragma unroll
    for (int j = 0; j < 6; ++j) a[j] = *reinterpret_cast<const f32x2*>(vb + (6 * wid + j) * (R_BT * 32));
  };

  // prologue: raw(0..2), U(0); transform raw(0); raw(3) (into raw(0)'s stage, after a barrier);
  // transform raw(1); operands of chunk 0. Per chunk each wave then issues exactly 9 U loads + 2 DMAs,
  // in that order (past-the-end fetches read chunk 0 / the zero block), so the counted vmcnt values
  // are exact. (the sched_barriers pin the issue order they rely on)
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(2, 2);
  __builtin_amdgcn_sched_barrier(0);
  load_u(0, uu[0]);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | 13);  // vmcnt(13): raw(0) landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  {
    float d[4][5];
    transform_read(0, d);
    if (jh == 0)
      transform_write(JH0{}, d, 0);
    else
      transform_write(JH1{}, d, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70 | 11);  // vmcnt(11): raw(1) landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();  // every wave has read raw stage 0
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(3, 0);
  __builtin_amdgcn_sched_barrier(0);
  {
    float d[4][5];
    transform_read(1, d);
    if (jh == 0)
      transform_write(JH0{}, d, 1);
    else
      transform_write(JH1{}, d, 1);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own V stores done
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_a(0, aa[0]);

  // chunk k: multiply V(k) (operands read during chunk k-1) by U(k); read V(k+1); transform raw(k+2)
  // into V stage (k+2) % 3; fetch U(k+1) and raw(k+4) (into raw(k+1)'s stage).
  auto step = [&](auto jh_c, int k, f32x4 (&uc)[3][3], f32x4 (&un)[3][3], f32x2 (&ac)[6], f32x2 (&an)[6])
                  __attribute__((always_inline)) {
    // vmcnt(2): U(k) and raw(k+2) landed (only raw(k+3) may be in flight); lgkmcnt(0): own V stores
    // and operand reads done
    __builtin_amdgcn_s_waitcnt(0x0070 | 2);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read_a((k + 1) % 3, an);
    float d[4][5];
    transform_read((k + 2) % 3, d);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)  // K step outermost: an accumulator's two MFMAs are 18 apart
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          acc[j][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][s2], uc[nt][j >> 1][(j & 1) * 2 + s2], acc[j][nt], 0,
                                                            0, 0);
    transform_write(jh_c, d, (k + 2) % 3);
    // U(k+1) (into the registers U(k-1) used) and raw(k+4) after the transform: the transform's
    // temporaries and the next U set do not overlap (register pressure), and U still has half a
    // chunk to arrive
    load_u(k + 1, un);
#pragma unroll
    for (int g = 0; g < 9; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // DS read (6 operand, 20 transform)
    }
#pragma unroll
    for (int g = 0; g < 10; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // VALU
    }
#pragma unroll
    for (int g = 0; g < 6; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);  // DS write
    }
#pragma unroll
    for (int g = 0; g < 9; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (9 U loads)
    }
    // raw(k+4) last, in a scheduling region of its own: every U load of this chunk is older than it,
    // which the counted vmcnt(2) at the next chunk's top relies on
    __builtin_amdgcn_sched_barrier(0);
    issue_raw(k + 4, (k + 1) % 3);
  };
  auto chunks = [&](auto jh_c) __attribute__((always_inline)) {
    if constexpr (NCH > 0) {
#pragma unroll
      for (int kk = 0; kk < NCH; ++kk) step(jh_c, kk, uu[kk & 1], uu[(kk + 1) & 1], aa[kk & 1], aa[(kk + 1) & 1]);
    } else {
      int k = 0;
      for (; k + 2 <= nchunk; k += 2) {
        step(jh_c, k, uu[0], uu[1], aa[0], aa[1]);
        step(jh_c, k + 1, uu[1], uu[0], aa[1], aa[0]);
      }
      if (k < nchunk) step(jh_c, k, uu[0], uu[1], aa[0], aa[1]);
    }
  };
  if (jh == 0)
    chunks(JH0{});
  else
    chunks(JH1{});
  __builtin_amdgcn_s_waitcnt(0x0F70);  // drain past-the-end fetches before LDS is reused

  // epilogue: unit = (tile, 4 channels, output column b); Z[i][b][tile][co] (48 KB) through LDS
  constexpr int CQ = 12, UNITS = R_BT * CQ * 4, UPT = UNITS / 256;
  static_assert(UNITS % 256 == 0, "epilogue units");
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  size_t u_o[UPT];
  int u_ok[UPT], u_z[UPT];
  f32x4 u_b[UPT], u_r[UPT][2];
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    const int un = tid + 256 * u;
    const int b = un & 3, rest = un >> 2;
    const int cq = rest % CQ, tl = rest / CQ;
    const int gp = pg0 + (tl >> 3);
    const bool live = gp < n_patches;
    const int gpc = live ? gp : pg0;
    const int f = gpc / (PY * PX), r = gpc - f * (PY * PX);
    const int pr = r / PX, pc = r - pr * PX;
    const int yy = pr * 8 + 2 * ((tl >> 1) & 3), xx = pc * 8 + 4 * (tl & 1) + b;
    const int co = n0 + 4 * cq;
    u_o[u] = ((size_t)(f * H + yy) * W + xx) * CO + co;
    u_z[u] = (b * R_BT + tl) * 48 + 4 * cq;
    u_ok[u] = live;
    u_b[u] = (p.bias && live) ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
      u_r[u][a2] = (res && live) ? *reinterpret_cast<const f32x4*>(res + u_o[u] + (size_t)a2 * W * CO)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float* zs = reinterpret_cast<float*>(smem);
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < 3; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) m[j] = acc[j][nt][r];
      const float d12 = m[1] - m[2], s12 = m[1] + m[2], d34 = m[3] - m[4], s34 = m[3] + m[4];
      const float z[4] = {m[0] + s12 + s34, d12 + 2.f * d34, s12 + 4.f * s34, d12 + 8.f * d34 + m[5]};
#pragma unroll
      for (int b = 0; b < 4; ++b) zs[((wid * 4 + b) * R_BT + 4 * q + r) * 48 + nt * 16 + l16] = z[b];
    }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    if (!u_ok[u]) continue;
    f32x4 z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = *reinterpret_cast<const f32x4*>(zs + i * 4 * R_BT * 48 + u_z[u]);
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2) {
      f32x4 v = (a2 == 0 ? z[0] + z[1] + z[2] : z[1] - z[2] - z[3]) + u_b[u];
      if (res) v += u_r[u][a2];
      if (p.relu) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
      }
      *reinterpret_cast<f32x4*>(yout + u_o[u] + (size_t)a2 * W * CO) = v;
    }
  }
}

template <int NCH>
hipError_t launch_r(const ConvParams& p, hipStream_t s) {
  const int n_patches = p.N * p.To * (p.Ho >> 3) * (p.Wo >> 3);
  const int n_co = p.Cout / 48;
  hipLaunchKernelGGL((conv_wino_r<NCH>), dim3(((n_patches + 1) / 2) * n_co), dim3(256), 0, s, p, n_co, n_patches);
  return hipGetLastError();
}

}  // namespace

bool winor_supported(const ConvParams& p) { return winoq_supported(p) && p.Ho % 8 == 0 && p.Wo % 8 == 0; }

// p.w: U[Cin/8][4][Cout][4][6][2] (winor_transform_weights).
hipError_t launch_winor(const ConvParams& p, hipStream_t s) {
  if (!winor_supported(p)) return hipErrorInvalidValue;
  switch (p.Cin >> 3) {
    case 8: return launch_r<8>(p, s);
    case 16: return launch_r<16>(p, s);
    default: return launch_r<0>(p, s);
  }
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: the product dispatch
hipError_t launch_winor_ko(const ConvParams& p, hipStream_t s, int ko) {
  (void)ko;
  return launch_winor(p, s);
}
#endif

// Host: U[c/8][i][o][(c%8)/2][j][c%2] = (G2 g G4^T)[i][j] in double, g = folded 3x3 kernel (rows = H).
void winor_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G2[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  static const double G4[6][3] = {{1.0 / 4, 0, 0},
                                  {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                  {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                  {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                  {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                  {0, 0, 1}};
  for (size_t i = 0; i < (size_t)24 * cin_p * cout_p; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* g = w + ((size_t)o * cin + c) * 9;
      double tmp[4][3];
      for (int i = 0; i < 4; ++i)
        for (int v = 0; v < 3; ++v) tmp[i][v] = G2[i][0] * g[0 * 3 + v] + G2[i][1] * g[1 * 3 + v] + G2[i][2] * g[2 * 3 + v];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 6; ++j) {
          const double u = tmp[i][0] * G4[j][0] + tmp[i][1] * G4[j][1] + tmp[i][2] * G4[j][2];
          U[((((size_t)(c / 8) * 4 + i) * cout_p + o) * 4 + (c % 8) / 2) * 12 + j * 2 + (c % 2)] = (float)u;
        }
    }
}
