// Implicit-GEMM 3-D convolution for the R(2+1)D-18 encoder on gfx950.
//
// Replaces the cuDNN conv3d + BatchNorm3d(eval) + ReLU (+ residual add) sequences of torchvision's
// r2plus1d_18 (stem, Conv2Plus1D spatial 1x3x3 / temporal 3x1x1, 1x1x1 downsample) called from
// src/model/R2plus1D_18_MotionNet.py:29-37, and the decoder's low-resolution 1x1x1 projections.
//
// Design (MI355X):
//  * activations channels-last [N][T][H][W][C], C padded so that one K step (16 fp32 / 32 bf16
//    channels = 64 B) lies inside one tap -> 64-B coalesced row segments; the im2col A tile is
//    gathered on the fly, never materialised;
//  * A and B tiles of each K step are copied global -> LDS by global_load_lds_dwordx4 (LDS-DMA, no
//    VGPR staging) into a 3-stage ring; per-wave counted s_waitcnt vmcnt + raw s_barrier;
//  * tile image: 64-B rows, 16-B slot q of row r stored at q ^ g[(r >> 2) & 3], g = {0, 2, 3, 1},
//    so every ds_read_b128 lane group hits 16 distinct bank quads; the swizzle is applied to the
//    per-lane DMA SOURCE address because DMA writes are lane-linear;
//  * fp32: v_mfma_f32_16x16x4_f32 (exact fp32), 4 MFMAs per 16-B slot with k permuted inside the
//    slot (MFMA j of lane group q uses k = 4q + j); bf16: v_mfma_f32_16x16x32_bf16, the slot is
//    exactly the lane's 8-element operand. fp32 accumulation either way;
//  * 1-D grid with an XCD-aware swizzle, N tiles fastest: the blocks re-reading one A tile (and the
//    3x3 halo rows of their neighbours) share an XCD's L2;
//  * the MFMAs compute D^T = W . A^T (weights as the A operand): an accumulator lane then holds 4
//    CONSECUTIVE output channels of one voxel, so the epilogue (folded-BN bias, residual add, ReLU)
//    moves 16-B fp32 / 8-B bf16 vectors instead of one element per lane (same products, same
//    accumulation order: bit-identical to the untransposed form).
#include <hip/hip_bf16.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

__device__ inline bf16x8 pack_bf16x8(f32x4 a, f32x4 b) {
  return bf16x8{(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3],
                (__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
}

// x = hi + mid + lo, each the bf16 (round to nearest) of the remainder: fp32's 24 bits in 3 pieces
__device__ inline void split3_bf16x8(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
  hi = pack_bf16x8(a, b);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] -= (float)hi[e];
    b[e] -= (float)hi[4 + e];
  }
  mid = pack_bf16x8(a, b);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] -= (float)mid[e];
    b[e] -= (float)mid[4 + e];
  }
  lo = pack_bf16x8(a, b);
}

__device__ inline int xcd_swizzle(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ inline f32x4 load_res4(const void* res, size_t o, int bf16) {
  if (bf16) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(res) + o);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
  return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(res) + o);
}

template <bool NTS = false>
__device__ inline void store_out4(void* y, size_t o, f32x4 v, int bf16) {
  if constexpr (NTS) {  // non-temporal (fp32 outputs only)
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(reinterpret_cast<float*>(y) + o));
    return;
  }
  if (bf16)
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(y) + o) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  else
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(y) + o) = v;
}

// acc[i][j] (D^T layout): lane (l16, q) holds channels n0 + 16j + 4q .. +3 of voxel m_base + 16i + l16.
// Cout is a multiple of 16, so a 4-channel group is either all inside or all outside. Each lane
// reads its residual vector before writing the same addresses (res may alias y).
// EF >= 0: the flags at compile time (bit 0 residual, 1 ReLU, 2 8-channel-blocked output; fp32 out),
// so only one form of each statement is in the code; EF < 0: read from p.
// Load order: every bias vector (and, where MT x NT <= 16, every residual vector) before the first
// store, then ONE explicit vmcnt(0). A load issued after a store is waited for with every older
// vector-memory op (vmcnt retires in order), and the compiler's own waits in the per-element
// branches were vmcnt(0): the per-element form paid the store latency once per (row, N tile) --
// MT x NT times per block. Bigger residual tiles load one row at a time (one wait per row).
template <int MT, int NT, int EF = -1, bool NTS = false>
__device__ inline void epilogue(const ConvParams& p, const f32x4 (&acc)[MT][NT], int m_base, int n0, int q, int l16) {
  const bool has_res = EF < 0 ? p.res != nullptr : (EF & 1) != 0;
  const bool relu = EF < 0 ? p.relu != 0 : (EF & 2) != 0;
  const bool c8 = EF < 0 ? p.y_c8 != 0 : (EF & 4) != 0;
  const int obf = EF < 0 ? p.out_bf16 : 0;
  constexpr bool ALL_ROWS = MT * NT <= 16;
  f32x4 bv[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + j * 16 + 4 * q;
    bv[j] = p.bias && n < p.Cout ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // channels-last, or 8-channel blocks [Cout/8][M][8] (p.y_c8, fp32)
  auto off = [&](int m, int n) { return c8 ? ((size_t)(n >> 3) * p.M + m) * 8 + (n & 7) : (size_t)m * p.Cout + n; };
  auto load_row = [&](int i, f32x4 (&r)[NT]) __attribute__((always_inline)) {
    const int m = m_base + i * 16 + l16;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + j * 16 + 4 * q;
      r[j] = m < p.M && n < p.Cout ? load_res4(p.res, off(m, n), obf) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x4 rv[ALL_ROWS ? MT : 1][NT];
  if constexpr (ALL_ROWS) {
    if (has_res) {
#pragma unroll
      for (int i = 0; i < MT; ++i) load_row(i, rv[i]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the epilogue's loads landed (no store issued yet)
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m_base + i * 16 + l16;
    f32x4 rr[NT];
    if (has_res) {
      if constexpr (ALL_ROWS) {
#pragma unroll
        for (int j = 0; j < NT; ++j) rr[j] = rv[i][j];
      } else {
        load_row(i, rr);
        __builtin_amdgcn_s_waitcnt(0x0F70);
      }
    }
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + j * 16 + 4 * q;
      if (n >= p.Cout) continue;
      f32x4 v = acc[i][j] + bv[j] + (has_res ? rr[j] : f32x4{0.f, 0.f, 0.f, 0.f});
      if (relu) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = relu1(v[c]);
      }
      store_out4<NTS>(p.y, off(m, n), v, obf);
    }
  }
}

// Split-K partial sums: acc as is (no bias, residual or ReLU), fp32 channels-last [M][Cout].
template <int MT, int NT>
__device__ inline void partial_store(const ConvParams& p, const f32x4 (&acc)[MT][NT], float* part, int m_base, int n0,
                                     int q, int l16) {
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m_base + i * 16 + l16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + j * 16 + 4 * q;
      if (n < p.Cout) *reinterpret_cast<f32x4*>(part + (size_t)m * p.Cout + n) = acc[i][j];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA implicit GEMM. T = float (K step 16) or __bf16 (K step 32). 4 waves along M (BM = 64*MT),
// BN = 16*NT, S-stage ring. Requires Cin (and Cin2) % (K step) == 0.
// Fast divisors of the output-voxel decode (m -> wo, ho, to, clip) and of the tile index.
struct DmaDivs {
  FastDiv wo, ho, to, nt;
};

// BUF (round 5, the bf16 engines' strided / 1x1x1 convs and projections): conv_dma_x3's buffer-offset
// DMAs (a row's tap-validity bits and first-tap byte offset once per block; an A DMA is a bit test and
// a select beside a scalar tap / channel offset, a B DMA a constant offset; out-of-range offsets read
// zeros), where dma_buf_ok holds
// KO (tools/convbench timing knock-outs, 0 in the product; results wrong otherwise): 4 no DMAs in the
// loop, 8 no waits / barriers, 16 no MFMAs
template <typename T, int MT, int NT, int S, bool BUF = false, int KO = 0>
__global__ __launch_bounds__(256) void conv_dma(ConvParams p, int n_tiles, DmaDivs dv) {
  constexpr int EPS = 16 / sizeof(T);  // elements per 16-B slot
  constexpr int BKE = 4 * EPS;         // K elements per step (one 64-B row)
  constexpr int BM = 64 * MT, BN = 16 * NT;
  constexpr int A_INS = BM / 16, B_INS = BN / 16, T_INS = A_INS + B_INS;
  // DMA slot j of wave w: j < A_PER -> A instruction w*A_PER + j; else B instruction w + 4*(j - A_PER)
  // (past B_INS: the sink). Every slot's kind is a compile-time constant, so the per-step issue code
  // has no branches on it (a wave-index-dependent kind made the compiler emit both paths per slot).
  constexpr int A_PER = A_INS / 4, B_PER = (B_INS + 3) / 4;
  constexpr int PER_WAVE = A_PER + B_PER;
  static_assert(A_INS % 4 == 0, "A rows split evenly over the 4 waves");
  constexpr int STAGE = T_INS * 1024;  // bytes per ring stage (16 rows x 64 B per DMA instruction)
  constexpr int JUNK = S * STAGE;      // 1 KB sink for the padding DMAs
  __shared__ __align__(16) char smem[S * STAGE + 1024];

  const T* x = reinterpret_cast<const T*>(p.x);
  const T* x2 = reinterpret_cast<const T*>(p.x2);
  const T* w = reinterpret_cast<const T*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_split = p.n_split > 1 ? p.n_split : 1;
  int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int n_tb = gridDim.x / n_split;  // output tiles
  const int split = tile / n_tb;
  tile -= split * n_tb;
  const int tq = fdiv(tile, dv.nt);
  const int m0 = tq * BM, n0 = (tile - tq * n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;
  constexpr int G[4] = {0, 2, 3, 1};

  // per-lane DMA descriptors: the lane writes row (lane >> 2), physical slot (lane & 3)
  const int drow = lane >> 2;
  const int dq = (lane & 3) ^ G[(drow >> 2) & 3];  // logical slot this lane fetches
  const T* d_wrow[PER_WAVE];
  int d_t[PER_WAVE], d_h[PER_WAVE], d_w[PER_WAVE], d_pix[PER_WAVE];  // A rows: tap-(0,0,0) input voxel
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int idx = j < A_PER ? wid * A_PER + j : A_INS + wid + 4 * (j - A_PER);
    d_t[j] = d_h[j] = d_w[j] = d_pix[j] = 0;
    d_wrow[j] = w;
    if (j < A_PER) {
      int m = m0 + idx * 16 + drow;
      const bool ok = m < p.M;
      if (!ok) m = 0;
      const int mw = fdiv(m, dv.wo), wo = m - mw * p.Wo;
      const int mh = fdiv(mw, dv.ho), ho = mw - mh * p.Ho;
      const int mt = fdiv(mh, dv.to), to = mh - mt * p.To;
      d_t[j] = ok ? to * p.st - p.pt : -(1 << 20);  // a row past M never passes the bounds test
      d_h[j] = ho * p.sh - p.ph;
      d_w[j] = wo * p.sw - p.pw;
      // linear input-voxel index of tap (0,0,0); may point outside when padded (never used then)
      d_pix[j] = ((mt * p.Ti + d_t[j]) * p.Hi + d_h[j]) * p.Wi + d_w[j];
    } else if (idx < T_INS) {
      d_wrow[j] = w + (size_t)(n0 + (idx - A_INS) * 16 + drow) * p.Kp + EPS * dq;
    }
  }
  const int khw = p.KH * p.KW;
  const int kmain = p.KT * khw * p.Cin;  // K columns from x; the rest (1x1 dual input) from x2

  // BUF: per A row the tap-validity bits and the byte offsets of its first tap's pixel (from x - padpix
  // pixels, so never negative for a valid tap) in x and x2, slot dq included; per B slot the byte
  // offset of its weight row
  constexpr unsigned ES = sizeof(T);
  unsigned a_vm[A_PER], a_bo[A_PER], a_bo2[A_PER], b_bo[PER_WAVE];
  const int padpix = (p.pt * p.Hi + p.ph) * p.Wi + p.pw;
  const size_t vox = (size_t)p.N * p.Ti * p.Hi * p.Wi;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      BUF ? const_cast<T*>(x - (size_t)padpix * p.Cin) : nullptr, (short)0, BUF ? (int)((vox + padpix) * p.Cin * ES) : 0,
      0x00020000);
  const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
      BUF && x2 ? const_cast<T*>(x2) : nullptr, (short)0, BUF && x2 ? (int)(vox * p.Cin2 * ES) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      BUF ? const_cast<T*>(w) : nullptr, (short)0, BUF ? (int)((size_t)p.Cout * p.Kp * ES) : 0, 0x00020000);
  if constexpr (BUF) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      unsigned vm = 0;
      for (int kt = 0; kt < p.KT; ++kt)
        for (int kh = 0; kh < p.KH; ++kh)
          for (int kw = 0; kw < p.KW; ++kw) {
            const int ti = d_t[j] + kt, hi = d_h[j] + kh, wi = d_w[j] + kw;
            const bool ok = ((unsigned)ti < (unsigned)p.Ti) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
            vm |= (ok ? 1u : 0u) << ((kt * p.KH + kh) * p.KW + kw);
          }
      a_vm[j] = vm;
      a_bo[j] = (unsigned)(d_pix[j] + padpix) * (unsigned)(p.Cin * ES) + 16u * (unsigned)dq;
      a_bo2[j] = (unsigned)d_pix[j] * (unsigned)(p.Cin2 * ES) + 16u * (unsigned)dq;
    }
#pragma unroll
    for (int j = A_PER; j < PER_WAVE; ++j) {
      const int idx = A_INS + wid + 4 * (j - A_PER);
      b_bo[j] = idx < T_INS ? (unsigned)(((size_t)(n0 + (idx - A_INS) * 16 + drow) * p.Kp + EPS * dq) * ES) : 0x80000000u;
    }
  }

  // split-K (p.n_split > 1): this block sums K steps [kb, ke) of its tile
  const int nk_all = p.Kp / BKE;
  const int kb = split * nk_all / n_split, ke = (split + 1) * nk_all / n_split;

  // K-step cursor (issue() is called for k_step = kb, kb + 1, ... in order): channel offset c0 inside
  // tap (kt, kh, kw) of input x, then of x2 -- advanced incrementally, where the per-step scalar
  // divisions of the closed form cost ~3 SALU instructions per MFMA (PMC, layer2 SP1); the closed
  // form once for the start
  int c_c0 = 0, c_kt = 0, c_kh = 0, c_kw = 0, c_tap_pix = 0;
  bool c_second = kmain == 0;
  if (kb > 0) {
    const int e0 = kb * BKE;
    if (e0 >= kmain) {
      c_second = true;
      c_c0 = e0 - kmain;
    } else {
      const int tap = e0 / p.Cin;
      c_c0 = e0 - tap * p.Cin;
      c_kw = tap % p.KW;
      c_kh = (tap / p.KW) % p.KH;
      c_kt = tap / khw;
      c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
    }
  }
  auto issue = [&](int k_step, int slot) {
    const int k0 = k_step * BKE;
    const bool second = c_second;
    const int cin = second ? p.Cin2 : p.Cin;
    const T* xb = second ? x2 : x;
    const int c0 = c_c0, kt = c_kt, kh = c_kh, kw = c_kw, tap_pix = c_tap_pix;
    c_c0 += BKE;
    if (c_c0 == cin) {
      c_c0 = 0;
      if (++c_kw == p.KW) {
        c_kw = 0;
        if (++c_kh == p.KH) {
          c_kh = 0;
          if (++c_kt == p.KT) c_kt = 0, c_second = true;
        }
      }
      c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
    }
    if constexpr (BUF) {
      const unsigned tap = (unsigned)((kt * p.KH + kh) * p.KW + kw);
      const unsigned soff = (unsigned)(tap_pix * cin + c0) * ES, sb = (unsigned)k0 * ES;
#pragma unroll
      for (int j = 0; j < PER_WAVE; ++j) {
        const int idx = j < A_PER ? wid * A_PER + j : A_INS + wid + 4 * (j - A_PER);
        char* dst = (idx < T_INS) ? smem + slot * STAGE + idx * 1024 : smem + JUNK;
        if (j < A_PER) {
          const unsigned off = ((a_vm[j] >> tap) & 1u) ? (second ? a_bo2[j] : a_bo[j]) : 0x80000000u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? x2r : xr, (__attribute__((address_space(3))) void*)dst, 16,
                                                   off, soff, 0, 0);
        } else {
          const unsigned bo = b_bo[j];  // (through a local: see conv_dma_x3)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)dst, 16, bo, sb, 0, 0);
        }
      }
      return;
    }
    const T* xc = xb + c0 + EPS * dq;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int idx = j < A_PER ? wid * A_PER + j : A_INS + wid + 4 * (j - A_PER);
      const void* src;
      if (j < A_PER) {
        const int ti = d_t[j] + kt, hi = d_h[j] + kh, wi = d_w[j] + kw;
        // bitwise &: short-circuit && became nested exec-masked branches
        const bool ok = ((unsigned)ti < (unsigned)p.Ti) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
        // element offset in 32 bits (a tensor has < 2^32 elements): one v_mul_lo_u32, where the
        // 64-bit product was two v_mad_u64_u32
        const unsigned e = (unsigned)(d_pix[j] + tap_pix) * (unsigned)cin;
        src = ok ? (const void*)(xc + (size_t)e) : p.zero;
      } else {
        src = idx < T_INS ? (const void*)(d_wrow[j] + k0) : p.zero;
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

  const int nk = ke - kb;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(kb + s, s);

  const int pq = q ^ G[l16 >> 2];  // physical slot of this lane's fragment reads
  const int a_off = (wid * 16 * MT + l16) * 64 + pq * 16;
  const int b_off = A_INS * 1024 + l16 * 64 + pq * 16;
  for (int k = 0; k < nk; ++k) {
    // stage k landed (this wave's DMAs), then every wave's (barrier); everyone is also done with
    // stage k-1, whose slot is refilled below.
    if constexpr ((KO & 8) == 0) {
      if (k + S - 2 < nk) {
        if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER_WAVE) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_WAVE) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((KO & 4) == 0)
      if (k + S - 1 < nk) issue(kb + k + S - 1, (k + S - 1) % S);
    const char* st = smem + (k % S) * STAGE;
    if constexpr (sizeof(T) == 4) {
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
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][kk], a[i][kk], acc[i][j], 0, 0, 0);
    } else {
      bf16x8 a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + a_off + i * 16 * 64);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(st + b_off + j * 16 * 64);
      if constexpr ((KO & 16) != 0) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j][0] += (float)a[i][j & 7] * (float)b[j][i & 7];
      } else {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  if (n_split > 1)
    partial_store<MT, NT>(p, acc, p.part + (size_t)split * p.M * p.Cout, m0 + wid * 16 * MT, n0, q, l16);
  else
    epilogue<MT, NT>(p, acc, m0 + wid * 16 * MT, n0, q, l16);
}

// ---------------------------------------------------------------------------------------------
// conv_dma_w (round 5, bf16 engines; Cin, Cin2 % 64 == 0): conv_dma<__bf16>'s implicit GEMM with
// 128-B LDS rows -- a ring stage holds two 32-deep K steps of each A / B row side by side, so every
// DMA row is a whole 128-B line of a tap's channels (conv_dma gathers 64-B half lines, and its
// strided convs are bound by that gather: profiles/r05aj_bf16_conv_dma_buffer_dmas.txt). A DMA
// instruction fills 8 rows (lane = row lane / 8, physical slot lane % 8, which holds logical slot
// phys ^ (row % 8): 8 consecutive lanes of a fragment read hit distinct banks). The buffer-offset
// DMAs of conv_dma's BUF form. Per stage the two K steps run in conv_dma's order (step 2s for
// every (i, j), then step 2s + 1), so the outputs are bit-identical to conv_dma's.
template <int MT, int NT, int S>
__global__ __launch_bounds__(256) void conv_dma_w(ConvParams p, int n_tiles, DmaDivs dv) {
  constexpr int BKE = 64;  // bf16 K elements per ring stage (one 128-B row)
  constexpr int BM = 64 * MT, BN = 16 * NT;
  constexpr int A_INS = BM / 8, B_INS = BN / 8, T_INS = A_INS + B_INS;  // DMA instructions (8 rows x 128 B)
  constexpr int A_PER = A_INS / 4, B_PER = (B_INS + 3) / 4;
  constexpr int PER_WAVE = A_PER + B_PER;
  static_assert(A_INS % 4 == 0, "A rows split evenly over the 4 waves");
  constexpr int STAGE = T_INS * 1024;
  constexpr int JUNK = S * STAGE;
  __shared__ __align__(16) char smem[S * STAGE + 1024];

  const __bf16* x = reinterpret_cast<const __bf16*>(p.x);
  const __bf16* x2 = reinterpret_cast<const __bf16*>(p.x2);
  const __bf16* w = reinterpret_cast<const __bf16*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tq = fdiv(tile, dv.nt);
  const int m0 = tq * BM, n0 = (tile - tq * n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;

  const int drow = lane >> 3;               // row of the instruction's 8
  const int dq = (lane & 7) ^ drow;         // logical 16-B slot this lane fetches (row % 8 = drow)
  constexpr unsigned ES = 2;
  const int padpix = (p.pt * p.Hi + p.ph) * p.Wi + p.pw;
  const size_t vox = (size_t)p.N * p.Ti * p.Hi * p.Wi;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(x - (size_t)padpix * p.Cin), (short)0, (int)((vox + padpix) * p.Cin * ES), 0x00020000);
  const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
      x2 ? const_cast<__bf16*>(x2) : nullptr, (short)0, x2 ? (int)(vox * p.Cin2 * ES) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(w), (short)0, (int)((size_t)p.Cout * p.Kp * ES), 0x00020000);
  unsigned a_vm[A_PER], a_bo[A_PER], a_bo2[A_PER], b_bo[B_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    int m = m0 + (wid * A_PER + j) * 8 + drow;
    const bool ok = m < p.M;
    if (!ok) m = 0;
    const int mw = fdiv(m, dv.wo), wo = m - mw * p.Wo;
    const int mh = fdiv(mw, dv.ho), ho = mw - mh * p.Ho;
    const int mt = fdiv(mh, dv.to), to = mh - mt * p.To;
    const int dt = ok ? to * p.st - p.pt : -(1 << 20), dh = ho * p.sh - p.ph, dw = wo * p.sw - p.pw;
    const int dpix = ((mt * p.Ti + dt) * p.Hi + dh) * p.Wi + dw;
    unsigned vm = 0;
    for (int kt = 0; kt < p.KT; ++kt)
      for (int kh = 0; kh < p.KH; ++kh)
        for (int kw = 0; kw < p.KW; ++kw) {
          const int ti = dt + kt, hi = dh + kh, wi = dw + kw;
          const bool v = ((unsigned)ti < (unsigned)p.Ti) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
          vm |= (v ? 1u : 0u) << ((kt * p.KH + kh) * p.KW + kw);
        }
    a_vm[j] = vm;
    a_bo[j] = (unsigned)(dpix + padpix) * (unsigned)(p.Cin * ES) + 16u * (unsigned)dq;
    a_bo2[j] = (unsigned)dpix * (unsigned)(p.Cin2 * ES) + 16u * (unsigned)dq;
  }
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int idx = wid + 4 * j;  // B instruction: rows 8 idx .. 8 idx + 7 of the N tile
    b_bo[j] = idx < B_INS ? (unsigned)(((size_t)(n0 + idx * 8 + drow) * p.Kp + 8 * dq) * ES) : 0x80000000u;
  }
  const int khw = p.KH * p.KW;
  const int kmain = p.KT * khw * p.Cin;
  int c_c0 = 0, c_kt = 0, c_kh = 0, c_kw = 0, c_tap_pix = 0;
  bool c_second = kmain == 0;
  auto issue = [&](int k_step, int slot) {
    const bool second = c_second;
    const int cin = second ? p.Cin2 : p.Cin;
    const int c0 = c_c0, kt = c_kt, kh = c_kh, kw = c_kw, tap_pix = c_tap_pix;
    c_c0 += BKE;
    if (c_c0 == cin) {
      c_c0 = 0;
      if (++c_kw == p.KW) {
        c_kw = 0;
        if (++c_kh == p.KH) {
          c_kh = 0;
          if (++c_kt == p.KT) c_kt = 0, c_second = true;
        }
      }
      c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
    }
    const unsigned tap = (unsigned)((kt * p.KH + kh) * p.KW + kw);
    const unsigned soff = (unsigned)(tap_pix * cin + c0) * ES, sb = (unsigned)(k_step * BKE) * ES;
    char* stg = smem + slot * STAGE;
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const unsigned off = ((a_vm[j] >> tap) & 1u) ? (second ? a_bo2[j] : a_bo[j]) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? x2r : xr,
                                               (__attribute__((address_space(3))) void*)(stg + (wid * A_PER + j) * 1024), 16,
                                               off, soff, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int idx = wid + 4 * j;
      char* dst = idx < B_INS ? stg + (A_INS + idx) * 1024 : smem + JUNK;
      const unsigned bo = b_bo[j];  // (through a local: see conv_dma_x3)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)dst, 16, bo, sb, 0, 0);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kp / BKE;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  // fragment rows: A row wid 16 MT + 16 i + l16, B row 16 j + l16 (both = l16 mod 8); slot (4 h + q)
  const int sw = l16 & 7;
  const int a_off = (wid * 16 * MT + l16) * 128, b_off = A_INS * 1024 + l16 * 128;
  for (int k = 0; k < nk; ++k) {
    if (k + S - 2 < nk) {
      if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER_WAVE) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (k + S - 1 < nk) issue(k + S - 1, (k + S - 1) % S);
    const char* st = smem + (k % S) * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int so = ((4 * h + q) ^ sw) * 16;
      bf16x8 a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + a_off + i * 16 * 128 + so);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(st + b_off + j * 16 * 128 + so);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
  }
  epilogue<MT, NT>(p, acc, m0 + wid * 16 * MT, n0, q, l16);
}

// ---------------------------------------------------------------------------------------------
// conv_dma_x3: the fp32 implicit GEMM on v_mfma_f32_16x16x32_bf16 with 3-way split operands.
// x = hi + mid + lo (each the bf16 of the remainder: fp32's 24 bits); the product is accumulated in
// fp32 as lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi (smallest first; the dropped terms are
// below 2^-24 of the product), i.e. fp32-accurate, at 6 x 16 instead of 8 x 32 MFMA cycles per
// 32-deep K block (2.67x the fp32 MFMA rate). The weights are split on the host into a bf16 image
// [Kp/32][3 pieces][Cout][32] (dma_x3_weight_image); the activations are LDS-DMA'd as fp32
// exactly as in conv_dma and split in registers.
//
// A ring stage holds one K pair = two 16-channel steps: A as two fp32 tiles of conv_dma's layout
// (64-B rows, swizzled slots), B as 3 pieces x BN rows of 64 B (32 bf16: slot q holds, for lane group
// q, k = 4q..4q+3 of the first step and of the second), so lane (l16, q) builds its 8-element bf16
// operands from its f32x4 slot of each step -- the same k set on both sides of the product.
// WN: waves along N (1: 4 waves x (BM/4 rows x BN); 2: 2 x 2 waves of (BM/2 rows x BN/2), halving the
// B-piece LDS reads per wave at twice the A splits).
// BUF (round 5; dma_x3_buf_ok: every tensor below 2^31 bytes, <= 31 taps): the DMAs as buffer loads
// with 32-bit offsets. A row's tap validity is a bit mask computed once per block and its pixel
// offset a per-row constant, so an A DMA costs 3 VALU (bit test, select of the row offset or an
// out-of-range offset, whose DMA reads zeros) beside a scalar tap / channel offset, and a B DMA
// none; the pointer form spent ~14 VALU per A DMA (bounds compares, 64-bit address, select) in a
// kernel whose split VALU already competes with the MFMAs for issue (profiles/r05q_dma_x3_knockouts.txt:
// no loop DMAs -25 % on layer2's 240-channel strided conv).
// KO (tools/convbench timing knock-outs, 0 in the product; results wrong otherwise): 1 no activation
// split (the fp32 bits reinterpreted as the three pieces), 2 no B-piece LDS reads, 4 no DMAs in the
// loop, 8 no waits / barriers, 16 no epilogue.
// WR (round 5, with BUF; Cin, Cin2 % 32 == 0 and an even step count): conv_dma_w's 128-B A rows -- a
// pixel's 32 channels of the pair in one LDS row (slots 0-3 the first step, 4-7 the second, XOR-swizzled
// by row % 8), so every A DMA row is a whole line; B, the products and their order are unchanged
// (bit-identical).
template <int MT, int NT, int S, int WN = 1, int EF = -1, int KO = 0, bool BUF = false, bool NTS = false, bool WR = false>
__global__ __launch_bounds__(256) void conv_dma_x3(ConvParams p, int n_tiles, DmaDivs dv) {
  static_assert(!WR || BUF, "128-B A rows use the buffer DMAs");
  static_assert(NT % WN == 0, "N tiles split evenly over the waves along N");
  constexpr int MTW = MT * WN, NTW = NT / WN;  // 16 x 16 tiles per wave
  constexpr int BM = 64 * MT, BN = 16 * NT;
  constexpr int A_INS = BM / 16, B_INS = 3 * NT;     // DMA instructions (16 rows x 64 B) per step / pair
  constexpr int A_PER = A_INS / 4, B_PER = (B_INS + 3) / 4;
  constexpr int PER_WAVE = 2 * A_PER + B_PER;
  static_assert(A_INS % 4 == 0, "A rows split evenly over the 4 waves");
  constexpr int A_BYTES = A_INS * 1024;
  constexpr int STAGE = (2 * A_INS + B_INS) * 1024;
  constexpr int JUNK = S * STAGE;  // 1 KB sink for the padding DMAs, when B_INS % 4 != 0
  constexpr int SINK = B_INS % 4 ? 1024 : 0;  // (N tile 128: 2 x 80 KB blocks per CU)
  __shared__ __align__(16) char smem[S * STAGE + SINK];

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* x2 = reinterpret_cast<const float*>(p.x2);
  const __bf16* w = reinterpret_cast<const __bf16*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_split = p.n_split > 1 ? p.n_split : 1;
  int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int n_tb = gridDim.x / n_split;
  const int split = tile / n_tb;
  tile -= split * n_tb;
  const int tq = fdiv(tile, dv.nt);
  const int m0 = tq * BM, n0 = (tile - tq * n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;
  constexpr int G[4] = {0, 2, 3, 1};

  const int nsteps = p.Kp / 16;           // 16-channel K steps
  const int npairs = (nsteps + 1) / 2;    // ring stages; an odd last step pairs with zeros
  const int drow = lane >> 2;
  const int dq = (lane & 3) ^ G[(drow >> 2) & 3];
  // A rows per lane: WR: 2 A_PER rows of 8 per instruction (row lane / 8), else A_PER rows of 16
  constexpr int RA = WR ? 2 * A_PER : A_PER;
  const int adq = WR ? (lane & 7) ^ (lane >> 3) : dq;  // logical A slot this lane fetches
  int d_t[RA], d_h[RA], d_w[RA], d_pix[RA];
#pragma unroll
  for (int j = 0; j < RA; ++j) {
    int m = WR ? m0 + (wid * RA + j) * 8 + (lane >> 3) : m0 + (wid * A_PER + j) * 16 + drow;
    const bool ok = m < p.M;
    if (!ok) m = 0;
    const int mw = fdiv(m, dv.wo), wo = m - mw * p.Wo;
    const int mh = fdiv(mw, dv.ho), ho = mw - mh * p.Ho;
    const int mt = fdiv(mh, dv.to), to = mh - mt * p.To;
    d_t[j] = ok ? to * p.st - p.pt : -(1 << 20);
    d_h[j] = ho * p.sh - p.ph;
    d_w[j] = wo * p.sw - p.pw;
    d_pix[j] = ((mt * p.Ti + d_t[j]) * p.Hi + d_h[j]) * p.Wi + d_w[j];
  }
  const __bf16* d_wrow[B_PER];
  unsigned b_bo[B_PER];  // BUF: byte offsets into the weight image
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int idx = wid + 4 * j;  // B instruction: piece idx / NT, rows 16 (idx % NT) ..
    const int pc = idx / NT, nr = idx - pc * NT;
    if constexpr (BUF)
      b_bo[j] = idx < B_INS ? (unsigned)((pc * p.Cout + n0 + nr * 16 + drow) * 64 + 16 * dq) : 0u;
    else
      d_wrow[j] = idx < B_INS ? w + ((size_t)pc * p.Cout + n0 + nr * 16 + drow) * 32 + 8 * dq : w;
  }
  // BUF: per A row, the tap-validity bits (tap = (kt KH + kh) KW + kw; 0 for a row past M) and the
  // byte offsets of its first tap's pixel in x and x2 (16-B slot dq included)
  unsigned a_vm[RA], a_bo[RA], a_bo2[RA];
  const int padpix = (p.pt * p.Hi + p.ph) * p.Wi + p.pw;  // the most negative first-tap pixel of a row
  const size_t vox = (size_t)p.N * p.Ti * p.Hi * p.Wi;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      BUF ? const_cast<float*>(x - (size_t)padpix * p.Cin) : nullptr, (short)0,
      BUF ? (int)((vox + padpix) * p.Cin * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
      BUF && x2 ? const_cast<float*>(x2) : nullptr, (short)0, BUF && x2 ? (int)(vox * p.Cin2 * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      BUF ? const_cast<__bf16*>(w) : nullptr, (short)0, BUF ? (int)((size_t)p.Cout * npairs * 192) : 0, 0x00020000);
  if constexpr (BUF) {
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      unsigned vm = 0;
      for (int kt = 0; kt < p.KT; ++kt)
        for (int kh = 0; kh < p.KH; ++kh)
          for (int kw = 0; kw < p.KW; ++kw) {
            const int ti = d_t[j] + kt, hi = d_h[j] + kh, wi = d_w[j] + kw;
            const bool ok = ((unsigned)ti < (unsigned)p.Ti) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
            vm |= (ok ? 1u : 0u) << ((kt * p.KH + kh) * p.KW + kw);
          }
      a_vm[j] = vm;
      // offsets from x - padpix pixels: never negative for a valid tap, so neither buffer offset wraps
      a_bo[j] = (unsigned)(d_pix[j] + padpix) * (unsigned)(p.Cin * 4) + 16u * (unsigned)adq;
      a_bo2[j] = (unsigned)d_pix[j] * (unsigned)(p.Cin2 * 4) + 16u * (unsigned)adq;
    }
  }
  const int khw = p.KH * p.KW;
  const int kmain = p.KT * khw * p.Cin;

  const int kb = split * npairs / n_split, ke = (split + 1) * npairs / n_split;
  int c_c0 = 0, c_kt = 0, c_kh = 0, c_kw = 0, c_tap_pix = 0;
  bool c_second = kmain == 0;
  if (kb > 0) {
    const int e0 = kb * 32;
    if (e0 >= kmain) {
      c_second = true;
      c_c0 = e0 - kmain;
    } else {
      const int tap = e0 / p.Cin;
      c_c0 = e0 - tap * p.Cin;
      c_kw = tap % p.KW;
      c_kh = (tap / p.KW) % p.KH;
      c_kt = tap / khw;
      c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
    }
  }
  auto issue = [&](int pair, int slot) {
    char* stg = smem + slot * STAGE;
    if constexpr (WR) {
      // both steps of the pair inside one tap of one input (Cin, Cin2 % 32): one cursor step of 32
      const bool second = c_second;
      const int cin = second ? p.Cin2 : p.Cin;
      const int c0 = c_c0, kt = c_kt, kh = c_kh, kw = c_kw, tap_pix = c_tap_pix;
      c_c0 += 32;
      if (c_c0 == cin) {
        c_c0 = 0;
        if (++c_kw == p.KW) {
          c_kw = 0;
          if (++c_kh == p.KH) {
            c_kh = 0;
            if (++c_kt == p.KT) c_kt = 0, c_second = true;
          }
        }
        c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
      }
      const unsigned tap = (unsigned)((kt * p.KH + kh) * p.KW + kw);
      const unsigned soff = (unsigned)(tap_pix * cin + c0) * 4u;
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        const unsigned off = ((a_vm[j] >> tap) & 1u) ? (second ? a_bo2[j] : a_bo[j]) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            second ? x2r : xr, (__attribute__((address_space(3))) void*)(stg + (wid * RA + j) * 1024), 16, off, soff, 0, 0);
      }
    }
#pragma unroll
    for (int sub = 0; sub < (WR ? 0 : 2); ++sub) {
      const bool valid = 2 * pair + sub < nsteps;  // wave-uniform
      const bool second = c_second;
      const int cin = second ? p.Cin2 : p.Cin;
      const float* xb = second ? x2 : x;
      const int c0 = c_c0, kt = c_kt, kh = c_kh, kw = c_kw, tap_pix = c_tap_pix;
      if (valid) {
        c_c0 += 16;
        if (c_c0 == cin) {
          c_c0 = 0;
          if (++c_kw == p.KW) {
            c_kw = 0;
            if (++c_kh == p.KH) {
              c_kh = 0;
              if (++c_kt == p.KT) c_kt = 0, c_second = true;
            }
          }
          c_tap_pix = (c_kt * p.Hi + c_kh) * p.Wi + c_kw;
        }
      }
      if constexpr (BUF) {
        // tap 31: no row's bit (<= 31 taps), the padding step of an odd K reads zeros
        const unsigned tap = valid ? (unsigned)((kt * p.KH + kh) * p.KW + kw) : 31u;
        const unsigned soff = (unsigned)(tap_pix * cin + c0) * 4u;
#pragma unroll
        for (int j = 0; j < A_PER; ++j) {
          const unsigned off = ((a_vm[j] >> tap) & 1u) ? (second ? a_bo2[j] : a_bo[j]) : 0x80000000u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              second ? x2r : xr, (__attribute__((address_space(3))) void*)(stg + sub * A_BYTES + (wid * A_PER + j) * 1024),
              16, off, soff, 0, 0);
        }
        continue;
      }
      const float* xc = xb + c0 + 4 * dq;
#pragma unroll
      for (int j = 0; j < A_PER; ++j) {
        const int ti = d_t[j] + kt, hi = d_h[j] + kh, wi = d_w[j] + kw;
        const bool ok = valid & ((unsigned)ti < (unsigned)p.Ti) & ((unsigned)hi < (unsigned)p.Hi) &
                        ((unsigned)wi < (unsigned)p.Wi);
        const unsigned e = (unsigned)(d_pix[j] + tap_pix) * (unsigned)cin;
        const void* src = ok ? (const void*)(xc + (size_t)e) : p.zero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(stg + sub * A_BYTES +
                                                                                   (wid * A_PER + j) * 1024),
                                         16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int idx = wid + 4 * j;
      char* dst = idx < B_INS ? stg + 2 * A_BYTES + idx * 1024 : smem + JUNK;
      if constexpr (BUF) {
        // (offsets through locals: a captured array element as the builtin's operand made the host-side
        // instantiation fail substitution)
        const unsigned bo = b_bo[j], so = (unsigned)pair * (unsigned)(192 * p.Cout);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)dst, 16, bo, so, 0, 0);
      } else {
        const void* src = idx < B_INS ? (const void*)(d_wrow[j] + (size_t)pair * 96 * p.Cout) : p.zero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
  };

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = ke - kb;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(kb + s, s);

  const int wm = wid % (4 / WN), wn = wid / (4 / WN);
  const int pq = q ^ G[l16 >> 2];
  const int a_off = (wm * 16 * MTW + l16) * 64 + pq * 16;
  const int b_off = 2 * A_BYTES + (wn * NTW) * 1024 + l16 * 64 + pq * 16;
  for (int k = 0; k < nk; ++k) {
    if constexpr ((KO & 8) == 0) {
      if (k + S - 2 < nk) {
        if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER_WAVE) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((KO & 4) == 0)
      if (k + S - 1 < nk) issue(kb + k + S - 1, (k + S - 1) % S);
    const char* st = smem + (k % S) * STAGE;
    bf16x8 ah[MTW], am[MTW], al[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      f32x4 a0, a1;
      if constexpr (WR) {
        const char* ar = st + (wm * 16 * MTW + i * 16 + l16) * 128;
        a0 = *reinterpret_cast<const f32x4*>(ar + ((q ^ (l16 & 7)) * 16));
        a1 = *reinterpret_cast<const f32x4*>(ar + (((4 + q) ^ (l16 & 7)) * 16));
      } else {
        a0 = *reinterpret_cast<const f32x4*>(st + a_off + i * 16 * 64);
        a1 = *reinterpret_cast<const f32x4*>(st + A_BYTES + a_off + i * 16 * 64);
      }
      if constexpr ((KO & 1) != 0) {
        ah[i] = __builtin_bit_cast(bf16x8, a0);
        am[i] = __builtin_bit_cast(bf16x8, a1);
        al[i] = ah[i];
      } else {
        split3_bf16x8(a0, a1, ah[i], am[i], al[i]);
      }
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      bf16x8 bh, bm, bl;
      if constexpr ((KO & 2) != 0) {
        bh = ah[0], bm = am[0], bl = al[0];
      } else {
        bh = *reinterpret_cast<const bf16x8*>(st + b_off + j * 1024);
        bm = *reinterpret_cast<const bf16x8*>(st + b_off + (NT + j) * 1024);
        bl = *reinterpret_cast<const bf16x8*>(st + b_off + (2 * NT + j) * 1024);
      }
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am[i], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah[i], c, 0, 0, 0);
      }
    }
  }
  if constexpr ((KO & 16) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) sum += acc[i][j][0] + acc[i][j][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  if (n_split > 1)
    partial_store<MTW, NTW>(p, acc, p.part + (size_t)split * p.M * p.Cout, m0 + wm * 16 * MTW, n0 + wn * 16 * NTW, q,
                            l16);
  else
    epilogue<MTW, NTW, EF, NTS>(p, acc, m0 + wm * 16 * MTW, n0 + wn * 16 * NTW, q, l16);
}

// ---------------------------------------------------------------------------------------------
// conv_proj_x3 (round 4): the decoder's 1x1x1 tap projections (P01 = W0 f_stem + W1 f_layer1, P2,
// P3: 64 output channels, K = 128 / 128 / 256) as a persistent split-bf16 GEMM. On conv_dma_x3 a
// 128-voxel block ran only K / 32 = 4 ring steps, so its prologue and epilogue latencies dominated
// (P01: 1.04 ms per 30 clips for 2.1 GB of traffic). Here each block DMAs W's three bf16 pieces to LDS
// once and its waves walk 32-voxel items of the map, loading the next item's activations (fp32,
// 16 B per lane and K block half) into registers while the current item's MFMAs run; the products,
// their order and the epilogue are conv_dma_x3's (bit-identical output).
//  * W image in LDS: [K/32][3 pieces][4 N tiles][16 rows][64 B], slot q of row r at q ^ G[r >> 2]
//    (the weight image of dma_x3_weight_image, re-sliced by LDS-DMA);
//  * item = 32 voxels (2 MFMA column blocks) x 64 channels: per K block 12 ds_read_b128, 8 f32x4
//    activation loads per lane, 48 MFMAs of 16 cycles.
template <int KB, int NB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv_proj_x3(ConvParams p, int n_items) {
  constexpr int G[4] = {0, 2, 3, 1};
  constexpr int PIECES = KB * 12;  // 1-KiB LDS pieces of W
  __shared__ __align__(16) char smem[PIECES * 1024];
  const float* x = reinterpret_cast<const float*>(p.x);
  const float* x2 = reinterpret_cast<const float*>(p.x2);
  const __bf16* w = reinterpret_cast<const __bf16*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;

  // W: piece j = (kb, pc, nt) holds rows 16 nt .. +15 of piece pc of K block kb; lane -> row lane / 4,
  // physical slot lane & 3 holding logical slot (lane & 3) ^ G[(row >> 2) & 3]
  {
    const int drow = lane >> 2, dq = (lane & 3) ^ G[(drow >> 2) & 3];
    for (int j = wid; j < PIECES; j += 4) {
      const int nt = j & 3, pc = (j >> 2) % 3, kb = j / 12;
      const __bf16* src = w + (((size_t)kb * 3 + pc) * p.Cout + 16 * nt + drow) * 32 + 8 * dq;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + j * 1024), 16, 0, 0);
    }
  }
  const int b_off = l16 * 64 + (q ^ G[l16 >> 2]) * 16;

  const int cin = p.Cin, cin2 = p.x2 ? p.Cin2 : 0;
  // activations of item it: voxel m = 32 it + 16 i + l16, K block kb, 16-channel half h: channels
  // 4q..4q+3 (conv_dma_x3's lane order); items past the end load nothing
  auto load_item = [&](int it, f32x4 (&a)[KB][2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = 32 * it + 16 * i + l16;
      const bool ok = it < n_items && m < p.M;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const bool second = 32 * kb >= cin;
        const float* src = second ? x2 + (size_t)m * cin2 + (32 * kb - cin) : x + (size_t)m * cin + 32 * kb;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (ok) v = *reinterpret_cast<const f32x4*>(src + 16 * h + 4 * q);
          a[kb][i][h] = v;
        }
      }
    }
  };
  auto compute = [&](int it, const f32x4 (&a)[KB][2][2]) __attribute__((always_inline)) {
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      bf16x8 ah[2], am[2], al[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) split3_bf16x8(a[kb][i][0], a[kb][i][1], ah[i], am[i], al[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const char* st = smem + (kb * 12 + j) * 1024 + b_off;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(st);
        const bf16x8 bm = *reinterpret_cast<const bf16x8*>(st + 4 * 1024);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(st + 8 * 1024);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          f32x4 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah[i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al[i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am[i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah[i], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am[i], c, 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah[i], c, 0, 0, 0);
        }
      }
    }
    epilogue<2, 4>(p, acc, 32 * it, 0, q, l16);
  };

  // NB register buffers: items it, it + S, .. it + (NB - 1) S in flight (S = waves in the grid);
  // the loop is unrolled NB times so every buffer index is a compile-time register
  const int S = gridDim.x * 4;
  int it = blockIdx.x * 4 + wid;
  f32x4 buf[NB][KB][2][2];
#pragma unroll
  for (int b = 0; b < NB - 1; ++b) load_item(it + b * S, buf[b]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the W DMAs landed
  __syncthreads();
  while (it < n_items) {
    bool done = false;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (!done) {
        load_item(it + (NB - 1) * S, buf[(b + NB - 1) % NB]);
        compute(it, buf[b]);
        it += S;
        done = it >= n_items;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Register-staged variant for the stem's 1x7x7 conv over 3 (padded 4) fp32 input channels: the
// 16-deep K slice spans 4 taps, decoded per float4. BM = 128, BN = 16*NT.
template <int NT>
__global__ __launch_bounds__(256) void conv_stem_f32(ConvParams p, int n_tiles) {
  constexpr int MT = 2, BM = 128, BN = 16 * NT, NTH = 256;
  constexpr int A4 = BM * 4, B4 = BN * 4;
  constexpr int AL = A4 / NTH, BL = (B4 + NTH - 1) / NTH;
  __shared__ f32x4 As[2][4][BM];
  __shared__ f32x4 Bs[2][4][BN];
  const float* x = reinterpret_cast<const float*>(p.x);
  const float* wt = reinterpret_cast<const float*>(p.w);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tile = xcd_swizzle(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;
  const int q = lane >> 4, l16 = lane & 15;

  int a_n[AL], a_t[AL], a_h[AL], a_w[AL], a_q[AL], a_r[AL];
  bool a_ok[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int e = tid + i * NTH;
    a_r[i] = e >> 2;
    a_q[i] = e & 3;
    int m = m0 + a_r[i];
    a_ok[i] = m < p.M;
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
  // the stem's geometry is fixed (launch_stem checks it): 1x7x7 taps over 4 (3 + pad) channels, so
  // a float4 K group is exactly one tap and the tap decode is a division by the constant 7
  constexpr int KW = 7, CIN = 4;
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int k = k0 + 4 * a_q[i];
      const int tap = k / CIN, kh = tap / KW, kw = tap - kh * KW;
      const int hi = a_h[i] + kh, wi = a_w[i] + kw;
      const bool ok = a_ok[i] && (k < p.K) && (unsigned)a_t[i] < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi &&
                      (unsigned)wi < (unsigned)p.Wi;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok) v = *reinterpret_cast<const f32x4*>(x + ((((size_t)a_n[i] * p.Ti + a_t[i]) * p.Hi + hi) * p.Wi + wi) * CIN);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * NTH;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < B4) v = *reinterpret_cast<const f32x4*>(wt + (size_t)(n0 + (e >> 2)) * p.Kp + k0 + 4 * (e & 3));
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i) As[buf][a_q[i]][a_r[i]] = ra[i];
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * NTH;
      if (e < B4) Bs[buf][e & 3][e >> 2] = rb[i];
    }
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = p.Kp / 16;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tiles((kt + 1) * 16);
    f32x4 a[MT], b[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) a[i] = As[cur][q][wid * 32 + i * 16 + l16];
#pragma unroll
    for (int j = 0; j < NT; ++j) b[j] = Bs[cur][q][j * 16 + l16];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][kk], a[i][kk], acc[i][j], 0, 0, 0);
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  epilogue<MT, NT>(p, acc, m0 + wid * 32, n0, q, l16);
}

// bf16 stem for BASELINE config[4] (torchvision R2Plus1dStem conv 1x7x7, stride (1,2,2), padding
// (0,3,3), 3 -> 45 (64) channels; called from src/model/R2plus1D_18_MotionNet.py:29): the fp32 kernel
// above runs this conv on fp32 MFMAs, with 64 output channels in bf16 mode. Here the 4-channel fp32
// clip and the weights are split into bf16 pairs (x = hi + lo) in registers / on the host and
// multiplied on v_mfma_f32_16x16x32_bf16 as hi.hi + hi.lo + lo.hi (~fp32 accuracy: the stem's
// rounding would otherwise reach every downstream mask; 3 bf16 MFMAs still cost 3/16 of one fp32):
//  * K order (kernel row kh, tap kw 0..7 with kw = 7 a zero weight, channel 0..3): one 32-deep K
//    step per kernel row, and a lane's 8-element A fragment (k group q = taps 2q, 2q+1) is two
//    horizontally adjacent input pixels = two 16-B loads, straight from global memory (L1/L2: the
//    stride-2 7x7 windows of neighbouring voxels overlap ~12x);
//  * the hi and lo 64 x 224 weight images (2 x 28 KB) are staged in LDS once per block, 16-B slots
//    swizzled by the row (conflict-free ds_read_b128);
//  * block = 4 waves x 4 m tiles = 256 output voxels x 64 channels per item; persistent (round 4): two
//    blocks per CU stage the 56 KB of weight images once and walk their XCD's contiguous item range
//    (as conv_stem_x3); D^T = W . A^T, so the epilogue (folded-BN bias, ReLU) stores 8-B bf16 vectors
//    of 4 consecutive channels.

__device__ inline bf16x8 stem_bf16x8(f32x4 a, f32x4 b) {
  return bf16x8{(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3],
                (__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv_stem_bf16(ConvParams p, int n_items) {
  constexpr int MT = 4, NT = 4, ROW = 7 * 64, IMG = 64 * ROW;  // LDS weight row: 7 K steps x 64 B
  __shared__ __align__(16) char ws[2 * IMG];                    // hi image, lo image
  const float* x = reinterpret_cast<const float*>(p.x);
  const char* w16 = reinterpret_cast<const char*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int q8 = n_items >> 3, r8 = n_items & 7, x8 = blockIdx.x & 7;  // gridDim.x % 8 == 0
  const int i_start = x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8;
  const int i_end = i_start + q8 + (x8 < r8 ? 1 : 0);
  const int i_step = gridDim.x >> 3;
  if (i_start + (int)(blockIdx.x >> 3) >= i_end) return;  // block-uniform, before the barrier
  for (int e = tid; e < 2 * 64 * 28; e += 256) {  // [img][co][kh][slot] 16-B pieces, slot ^ (co & 3)
    const int im = e / (64 * 28), r0 = e - im * (64 * 28);
    const int co = r0 / 28, r = r0 - co * 28, kh = r >> 2, sl = r & 3;
    *reinterpret_cast<uint4*>(ws + im * IMG + co * ROW + kh * 64 + ((sl ^ (co & 3)) << 4)) =
        *reinterpret_cast<const uint4*>(w16 + (size_t)im * 64 * 448 + (size_t)co * 448 + kh * 64 + sl * 16);
  }
  __syncthreads();
  const int b_rd = l16 * ROW + ((q ^ (l16 & 3)) << 4);
  // the bias vectors once per block, not per item: a load issued after an item's stores would wait
  // for them (vmcnt retires in order)
  f32x4 bv[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) bv[j] = *reinterpret_cast<const f32x4*>(p.bias + 16 * j + 4 * q);
#pragma unroll 1
  for (int item = i_start + (int)(blockIdx.x >> 3); item < i_end; item += i_step) {
    const int m0 = item * 256 + wid * 64;
    // per m tile: input row of kh = 0 and the lane's first column (taps 2q, 2q+1)
    const float* rowp[MT];
    int hi0[MT], wi0[MT];
    bool live[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      int m = m0 + 16 * i + l16;
      live[i] = m < p.M;
      if (!live[i]) m = 0;
      const int wo = m % p.Wo;
      m /= p.Wo;
      const int ho = m % p.Ho;
      const int nt = m / p.Ho;  // n * To + t (stride 1 in time, no temporal padding)
      hi0[i] = 2 * ho - 3;
      wi0[i] = 2 * wo - 3 + 2 * q;
      rowp[i] = x + ((size_t)nt * p.Hi * p.Wi) * 4;
    }
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kh = 0; kh < 7; ++kh) {
      bf16x8 ah[MT], al[MT], bh[NT], bl[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int hi = hi0[i] + kh;
        const bool rok = live[i] && (unsigned)hi < (unsigned)p.Hi;
        const float* px = rowp[i] + ((size_t)hi * p.Wi + wi0[i]) * 4;
        f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
        if (rok && (unsigned)wi0[i] < (unsigned)p.Wi) v0 = *reinterpret_cast<const f32x4*>(px);
        if (rok && (unsigned)(wi0[i] + 1) < (unsigned)p.Wi) v1 = *reinterpret_cast<const f32x4*>(px + 4);
        ah[i] = stem_bf16x8(v0, v1);
        f32x4 r0, r1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r0[e] = v0[e] - (float)ah[i][e];
          r1[e] = v1[e] - (float)ah[i][4 + e];
        }
        al[i] = stem_bf16x8(r0, r1);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(ws + j * 16 * ROW + kh * 64 + b_rd);
        bl[j] = *reinterpret_cast<const bf16x8*>(ws + IMG + j * 16 * ROW + kh * 64 + b_rd);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], acc[i][j], 0, 0, 0);
        }
    }
    __bf16* y = reinterpret_cast<__bf16*>(p.y);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (!live[i]) continue;
      const size_t m = (size_t)m0 + 16 * i + l16;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + 4 * q;
        f32x4 v = acc[i][j] + bv[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = relu1(v[e]);
        *reinterpret_cast<bf16x4*>(y + m * 64 + n) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      }
    }
  }
}

// conv_dma's buffer-offset DMAs (BUF): the input from padpix pixels before its start, the second input
// and the weights below 2^31 bytes, the tap mask in 32 bits, and the bf16 engines only -- the fp32 form
// of conv_dma is a variant / fallback path (CLASFV_VARIANT_NO_DMA_BUF: the pointer form everywhere)
bool dma_buf_ok(const ConvParams& p, size_t es) {
  if ((p.vflags & CLASFV_VARIANT_NO_DMA_BUF) || es != 2) return false;
  const size_t lim = (size_t)1 << 31;
  const size_t vox = (size_t)p.N * p.Ti * p.Hi * p.Wi;
  const size_t padpix = ((size_t)p.pt * p.Hi + p.ph) * p.Wi + p.pw;
  return p.KT * p.KH * p.KW <= 32 && (vox + padpix) * p.Cin * es < lim && (!p.x2 || vox * p.Cin2 * es < lim) &&
         (size_t)p.Cout * p.Kp * es < lim;
}

// conv_dma_w (128-B rows): bf16, every K step inside one tap of one input (Cin, Cin2 % 64), one K
// range, the buffer-DMA limits (CLASFV_VARIANT_NO_DMA_W: conv_dma)
bool dma_w_ok_(const ConvParams& p) {
  if (p.vflags & CLASFV_VARIANT_NO_DMA_W) return false;
  if (!p.in_bf16 || p.stem || p.n_split > 1 || !dma_buf_ok(p, 2)) return false;
  return p.Cin % 64 == 0 && (!p.x2 || p.Cin2 % 64 == 0) && p.Kp == p.K && p.Kp % 64 == 0;
}

template <int MT, int NT, int S>
hipError_t launch_dma_w(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  const DmaDivs dv{fast_div(p.Wo), fast_div(p.Ho), fast_div(p.To), fast_div(nt)};
  hipLaunchKernelGGL((conv_dma_w<MT, NT, S>), dim3(mt * nt), dim3(256), 0, s, p, nt, dv);
  return hipGetLastError();
}

template <typename T, int MT, int NT, int S>
hipError_t launch_dma(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  const DmaDivs dv{fast_div(p.Wo), fast_div(p.Ho), fast_div(p.To), fast_div(nt)};
  const int n_split = p.n_split > 1 ? p.n_split : 1;
  if constexpr (sizeof(T) == 2 && MT == 2)
    if (dma_w_ok_(p)) return launch_dma_w<MT, NT, 2>(p, s);
  if (dma_buf_ok(p, sizeof(T)))
    hipLaunchKernelGGL((conv_dma<T, MT, NT, S, true>), dim3(mt * nt * n_split), dim3(256), 0, s, p, nt, dv);
  else
    hipLaunchKernelGGL((conv_dma<T, MT, NT, S>), dim3(mt * nt * n_split), dim3(256), 0, s, p, nt, dv);
  if (n_split > 1) return launch_split_sum(p, s);
  return hipGetLastError();
}

// conv_dma_x3's buffer-offset DMAs (BUF): every byte offset they form stays below 2^31 (the input
// from padpix pixels before its start, the second input, the weight image of rows_alloc rows) and
// the tap mask fits 31 bits (CLASFV_VARIANT_NO_DMA_BUF: the pointer form everywhere)
bool dma_x3_buf_ok(const ConvParams& p, int rows_alloc) {
  if (p.vflags & CLASFV_VARIANT_NO_DMA_BUF) return false;
  const size_t lim = (size_t)1 << 31;
  const size_t vox = (size_t)p.N * p.Ti * p.Hi * p.Wi;
  const size_t padpix = ((size_t)p.pt * p.Hi + p.ph) * p.Wi + p.pw;
  const int npairs = (p.Kp / 16 + 1) / 2;
  return p.KT * p.KH * p.KW <= 31 && (vox + padpix) * p.Cin * 4 < lim && (!p.x2 || vox * p.Cin2 * 4 < lim) &&
         (size_t)rows_alloc * npairs * 192 < lim;
}

template <int MT, int NT, int S, int WN = 1>
hipError_t launch_dma_x3_t(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  const DmaDivs dv{fast_div(p.Wo), fast_div(p.Ho), fast_div(p.To), fast_div(nt)};
  const int n_split = p.n_split > 1 ? p.n_split : 1;
  const dim3 grid(mt * nt * n_split);
  // the epilogue flags at compile time (split-K partials ignore them); the buffer-offset DMAs where
  // every tensor fits them
  const int ef = n_split > 1 ? 0 : (p.res ? 1 : 0) | (p.relu ? 2 : 0) | (p.y_c8 ? 4 : 0);
  // (round 5 A/B forms not in the library: non-temporal output stores ±0 in the forward,
  // profiles/r05ac_nt_stores_ab2.txt; 128-B A rows, bit-identical but 4.31 -> 4.37 ms per forward,
  // profiles/r05aq_dma_x3_wide_rows.txt -- the split-bf16 loop is not gather-bound enough for
  // whole-line rows to pay for the doubled per-lane row state)
  switch (dma_x3_buf_ok(p, nt * BN) ? ef + 8 : ef) {
    case 0: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 0>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 1: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 1>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 2: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 2>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 3: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 3>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 8: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 0, 0, true>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 9: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 1, 0, true>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 10: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 2, 0, true>), grid, dim3(256), 0, s, p, nt, dv); break;
    case 11: hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, 3, 0, true>), grid, dim3(256), 0, s, p, nt, dv); break;
    default:
      if (ef >= 8 || ef < 4) return hipErrorInvalidValue;
      if (dma_x3_buf_ok(p, nt * BN))
        hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN, -1, 0, true>), grid, dim3(256), 0, s, p, nt, dv);
      else
        hipLaunchKernelGGL((conv_dma_x3<MT, NT, S, WN>), grid, dim3(256), 0, s, p, nt, dv);
      break;
  }
  if (n_split > 1) return launch_split_sum(p, s);
  return hipGetLastError();
}

template <int NT>
hipError_t launch_stem(const ConvParams& p, hipStream_t s) {
  if (p.Cin != 4 || p.KT != 1 || p.KH != 7 || p.KW != 7) return hipErrorInvalidValue;  // conv_stem_f32's geometry
  const int mt = (p.M + 127) / 128, nt = (p.Cout + 16 * NT - 1) / (16 * NT);
  hipLaunchKernelGGL((conv_stem_f32<NT>), dim3(mt * nt), dim3(256), 0, s, p, nt);
  return hipGetLastError();
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip (CB_BF16 direct convs, ko 7300 + KO): conv_dma<__bf16, 2, NT, 3> knock-outs with
// the buffer DMAs (KO & 1: the pointer form)
template <int NT, int KO>
hipError_t dma_ko_t(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 128, BN = 16 * NT;
  const int mt = (p.M + BM - 1) / BM, nt = (p.Cout + BN - 1) / BN;
  const DmaDivs dv{fast_div(p.Wo), fast_div(p.Ho), fast_div(p.To), fast_div(nt)};
  hipLaunchKernelGGL((conv_dma<__bf16, 2, NT, 3, (KO & 1) == 0, KO & ~1>), dim3(mt * nt), dim3(256), 0, s, p, nt, dv);
  return hipGetLastError();
}
template <int NT>
hipError_t dma_ko_n(const ConvParams& p, int ko, hipStream_t s) {
  switch (ko) {
    case 0: return dma_ko_t<NT, 0>(p, s);
    case 1: return dma_ko_t<NT, 1>(p, s);
    case 4: return dma_ko_t<NT, 4>(p, s);
    case 8: return dma_ko_t<NT, 8>(p, s);
    case 16: return dma_ko_t<NT, 16>(p, s);
    case 12: return dma_ko_t<NT, 12>(p, s);
    case 28: return dma_ko_t<NT, 28>(p, s);
  }
  return hipErrorInvalidValue;
}
hipError_t dma_bf16_ko(const ConvParams& p, int bn, int ko, hipStream_t s) {
  if (ko == 100 || ko == 101) {  // conv_dma_w, 2 / 3 ring stages
    if (!dma_w_ok_(p)) return hipErrorInvalidValue;
    switch (bn) {
      case 64: return ko == 100 ? launch_dma_w<2, 4, 2>(p, s) : launch_dma_w<2, 4, 3>(p, s);
      case 96: return ko == 100 ? launch_dma_w<2, 6, 2>(p, s) : launch_dma_w<2, 6, 3>(p, s);
      case 128: return ko == 100 ? launch_dma_w<2, 8, 2>(p, s) : launch_dma_w<2, 8, 3>(p, s);
    }
    return hipErrorInvalidValue;
  }
  if (!p.in_bf16 || p.n_split > 1) return hipErrorInvalidValue;
  switch (bn) {
    case 64: return dma_ko_n<4>(p, ko, s);
    case 96: return dma_ko_n<6>(p, ko, s);
    case 128: return dma_ko_n<8>(p, ko, s);
  }
  return hipErrorInvalidValue;
}
#endif

template <typename T>
hipError_t launch_typed(const ConvParams& p, int bn, hipStream_t s) {
  switch (bn) {
    case 48: return launch_dma<T, 2, 3, 3>(p, s);
    case 64: return launch_dma<T, 2, 4, 3>(p, s);
    case 80: return launch_dma<T, 2, 5, 3>(p, s);
    case 96: return launch_dma<T, 2, 6, 3>(p, s);
    case 128: return launch_dma<T, 2, 8, 3>(p, s);
    case 144: return launch_dma<T, 2, 9, 3>(p, s);
  }
  return hipErrorInvalidValue;
}

#ifdef CLASFV_KNOCKOUTS
// (convbench CB_MT=4 only) bf16 with BM = 256 (4 waves x 64 rows): a K step moves (16 + NT) KiB for
// 16*NT MFMAs per wave instead of (8 + NT) KiB for 8*NT; measured slower than conv_dma_w's BM 128
// (0.48-0.50 vs 0.435 ms on layer2's strided conv, profiles/r05aj_bf16_conv_dma_buffer_dmas.txt)
hipError_t launch_bf16_m4(const ConvParams& p, int bn, hipStream_t s) {
  switch (bn) {
    case 48: return launch_dma<__bf16, 4, 3, 3>(p, s);
    case 64: return launch_dma<__bf16, 4, 4, 3>(p, s);
    case 80: return launch_dma<__bf16, 4, 5, 3>(p, s);
    case 96: return launch_dma<__bf16, 4, 6, 3>(p, s);
    case 128: return launch_dma<__bf16, 4, 8, 3>(p, s);
    case 144: return launch_dma<__bf16, 4, 9, 3>(p, s);
  }
  return hipErrorInvalidValue;
}
#endif

// fp32-engine stem on split-bf16 MFMAs (conv_stem_x3): conv_stem_bf16's structure and K order with
// three bf16 pieces per operand (x = hi + mid + lo, fp32's 24 bits) and the six products of
// conv_dma_x3, fp32 accumulation, 48 output channels (45 + 3 zero), fp32 output through the shared
// epilogue (channels-last or 8-channel-blocked for the temporal Winograd after it). Weights: hi, mid
// and lo images [48][7 kh][8 kw][4 c] bf16 (engine.hip, clasfv_finalize).
// Persistent over 256-voxel items (n_items): the three weight images are staged in LDS once per block
// and XCD x's blocks walk its contiguous item range with a stride of the blocks per XCD (gridDim.x % 8
// == 0), the one-item form's dispatch order.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv_stem_x3(ConvParams p, int n_items) {
  constexpr int MT = 4, NT = 3, CO = 16 * NT, ROW = 7 * 64, IMG = CO * ROW;
  __shared__ __align__(16) char ws[3 * IMG];  // hi, mid, lo images
  const float* x = reinterpret_cast<const float*>(p.x);
  const char* w16 = reinterpret_cast<const char*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int q8 = n_items >> 3, r8 = n_items & 7, x8 = blockIdx.x & 7;
  const int i_start = x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8;
  const int i_end = i_start + q8 + (x8 < r8 ? 1 : 0);
  const int i_step = gridDim.x >> 3;
  if (i_start + (int)(blockIdx.x >> 3) >= i_end) return;  // block-uniform, before the barrier
  for (int e = tid; e < 3 * CO * 28; e += 256) {  // [img][co][kh][slot] 16-B pieces, slot ^ (co & 3)
    const int im = e / (CO * 28), r0 = e - im * (CO * 28);
    const int co = r0 / 28, r = r0 - co * 28, kh = r >> 2, sl = r & 3;
    *reinterpret_cast<uint4*>(ws + im * IMG + co * ROW + kh * 64 + ((sl ^ (co & 3)) << 4)) =
        *reinterpret_cast<const uint4*>(w16 + (size_t)im * CO * 448 + (size_t)co * 448 + kh * 64 + sl * 16);
  }
  __syncthreads();
  const int b_rd = l16 * ROW + ((q ^ (l16 & 3)) << 4);
#pragma unroll 1
  for (int item = i_start + (int)(blockIdx.x >> 3); item < i_end; item += i_step) {
  const int m0 = item * 256 + wid * 64;
  const float* rowp[MT];
  int hi0[MT], wi0[MT];
  bool live[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int m = m0 + 16 * i + l16;
    live[i] = m < p.M;
    if (!live[i]) m = 0;
    const int wo = m % p.Wo;
    m /= p.Wo;
    const int ho = m % p.Ho;
    const int nt = m / p.Ho;  // n * To + t (stride 1 in time, no temporal padding)
    hi0[i] = 2 * ho - 3;
    wi0[i] = 2 * wo - 3 + 2 * q;
    rowp[i] = x + ((size_t)nt * p.Hi * p.Wi) * 4;
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kh = 0; kh < 7; ++kh) {
    bf16x8 ah[MT], am[MT], al[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int hi = hi0[i] + kh;
      const bool rok = live[i] && (unsigned)hi < (unsigned)p.Hi;
      const float* px = rowp[i] + ((size_t)hi * p.Wi + wi0[i]) * 4;
      f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
      if (rok && (unsigned)wi0[i] < (unsigned)p.Wi) v0 = *reinterpret_cast<const f32x4*>(px);
      if (rok && (unsigned)(wi0[i] + 1) < (unsigned)p.Wi) v1 = *reinterpret_cast<const f32x4*>(px + 4);
      split3_bf16x8(v0, v1, ah[i], am[i], al[i]);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(ws + j * 16 * ROW + kh * 64 + b_rd);
      const bf16x8 bm = *reinterpret_cast<const bf16x8*>(ws + IMG + j * 16 * ROW + kh * 64 + b_rd);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(ws + 2 * IMG + j * 16 * ROW + kh * 64 + b_rd);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am[i], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah[i], c, 0, 0, 0);
      }
    }
  }
  epilogue<MT, NT>(p, acc, m0, 0, q, l16);
  }  // items
}

}  // namespace

bool dma_w_ok(const ConvParams& p) { return dma_w_ok_(p); }

#ifdef CLASFV_KNOCKOUTS
hipError_t launch_dma_bf16_ko(const ConvParams& p, int bn, int ko, hipStream_t s) { return dma_bf16_ko(p, bn, ko, s); }
#endif

// conv_proj_x3: fp32 1x1x1 stride-1 convs to 64 channels over K = Cin (+ Cin2) = 128, both inputs
// multiples of 32 channels, channels-last in and out, no split-K (the decoder projections P01 and P2;
// K = 256 (P3) needs more registers than the item ring leaves and stays on conv_dma_x3). A split-bf16
// kernel: the no_dma_x3 variant (every non-stem GEMM on f32 MFMAs) excludes it too.
bool proj_x3_supported(const ConvParams& p) {
  if (p.vflags & CLASFV_VARIANT_NO_DMA_X3) return false;
  if (p.in_bf16 || p.out_bf16 || p.stem || p.x_c8 || p.y_c8 || p.n_split > 1) return false;
  if (p.KT != 1 || p.KH != 1 || p.KW != 1 || p.st != 1 || p.sh != 1 || p.sw != 1) return false;
  if (p.Cout != 64 || p.Cin % 32 || (p.x2 && p.Cin2 % 32)) return false;
  const int k = p.Cin + (p.x2 ? p.Cin2 : 0);
  if (p.Kp != k || k != 128) return false;
  return (size_t)p.M * (p.Cin > 64 ? p.Cin : 64) < ((size_t)1 << 31);
}

// p.w: dma_x3_weight_image of the conv (the same image conv_dma_x3 reads)
hipError_t launch_proj_x3(const ConvParams& p, hipStream_t s) {
  if (!proj_x3_supported(p)) return hipErrorInvalidValue;
  const int n_items = (p.M + 31) / 32;
  const int kb = p.Kp / 32;
  // persistent: one block (one wave per SIMD, 512 registers for the in-flight items) per CU, or
  // fewer when the map is small
  int blocks = 256;
  if (blocks * 4 > n_items) blocks = (n_items + 3) / 4;
  (void)kb;
  hipLaunchKernelGGL((conv_proj_x3<4, 3>), dim3(blocks), dim3(256), 0, s, p, n_items);
  return hipGetLastError();
}

// conv_dma_x3 (fp32 engines, non-stem implicit-GEMM convs): fp32 activations in, fp32 out
bool dma_x3_supported(const ConvParams& p) {
  return !(p.vflags & CLASFV_VARIANT_NO_DMA_X3) && !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x_c8 && !p.y_c8 &&
         p.Kp % 16 == 0 && p.Cin % 16 == 0 && (!p.x2 || p.Cin2 % 16 == 0) && p.Cout % 16 == 0;
}

// N tile of conv_dma_x3: the widest 16*NT (NT = 8 or <= 6: a stage is (16 MT + 3 NT) KiB, two per
// block, two blocks per CU) dividing Cout
int dma_x3_bn(int cout_p) {
  const int n16 = cout_p / 16;
  for (int c : {8, 6, 5, 4, 3})
    if (n16 % c == 0) return 16 * c;
  return 16 * (n16 % 2 == 0 ? 2 : 1);
}

hipError_t launch_dma_x3(const ConvParams& p, int bn, hipStream_t s) {
  if (!dma_x3_supported(p)) return hipErrorInvalidValue;
  switch (bn) {
    case 16: return launch_dma_x3_t<2, 1, 2>(p, s);
    case 32: return launch_dma_x3_t<2, 2, 2>(p, s);
    case 48: return launch_dma_x3_t<2, 3, 2>(p, s);
    case 64: return launch_dma_x3_t<2, 4, 2>(p, s);
    case 80: return launch_dma_x3_t<2, 5, 2>(p, s);
    case 96: return launch_dma_x3_t<2, 6, 2>(p, s);
    case 128: return launch_dma_x3_t<2, 8, 2>(p, s);
  }
  return hipErrorInvalidValue;
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: conv_dma_x3 tile / ring experiments (M tile 64*mt, N tile 16*nt, S stages)
hipError_t launch_dma_x3_cfg(const ConvParams& p, int mt, int nt, int S, hipStream_t s) {
  const int wn = getenv("CB_X3WN") ? atoi(getenv("CB_X3WN")) : 1;
  const int key = (wn == 2 ? 1000 : 0) + mt * 100 + nt * 10 + S;
  switch (key) {
    case 1242: return launch_dma_x3_t<2, 4, 2, 2>(p, s);
    case 1262: return launch_dma_x3_t<2, 6, 2, 2>(p, s);
    case 1282: return launch_dma_x3_t<2, 8, 2, 2>(p, s);
    case 1162: return launch_dma_x3_t<1, 6, 2, 2>(p, s);
    case 132: return launch_dma_x3_t<1, 3, 2>(p, s);
    case 133: return launch_dma_x3_t<1, 3, 3>(p, s);
    case 162: return launch_dma_x3_t<1, 6, 2>(p, s);
    case 163: return launch_dma_x3_t<1, 6, 3>(p, s);
    case 233: return launch_dma_x3_t<2, 3, 3>(p, s);
    case 243: return launch_dma_x3_t<2, 4, 3>(p, s);
    case 263: return launch_dma_x3_t<2, 6, 3>(p, s);
    case 432: return launch_dma_x3_t<4, 3, 2>(p, s);
    case 462: return launch_dma_x3_t<4, 6, 2>(p, s);
    case 152: return launch_dma_x3_t<1, 5, 2>(p, s);
    case 452: return launch_dma_x3_t<4, 5, 2>(p, s);
    case 253: return launch_dma_x3_t<2, 5, 3>(p, s);
    case 442: return launch_dma_x3_t<4, 4, 2>(p, s);
    case 482: return launch_dma_x3_t<4, 8, 2>(p, s);
    case 182: return launch_dma_x3_t<1, 8, 2>(p, s);
  }
  return launch_dma_x3(p, 16 * nt, s);
}

template <int NT, int KO>
static hipError_t dma_x3_ko_t(const ConvParams& p, hipStream_t s) {
  const int mt = (p.M + 127) / 128, nt = (p.Cout + 16 * NT - 1) / (16 * NT);
  const DmaDivs dv{fast_div(p.Wo), fast_div(p.Ho), fast_div(p.To), fast_div(nt)};
  hipLaunchKernelGGL((conv_dma_x3<2, NT, 2, 1, 2, (KO & 31), (KO & 32) != 0>), dim3(mt * nt), dim3(256), 0, s, p, nt, dv);
  return hipGetLastError();
}
// conv_dma_x3 knock-outs (KO bits of conv_dma_x3; + 32: the BUF form) at MT 2, 2 stages, the ReLU
// epilogue, N tile 16 nt
hipError_t launch_dma_x3_ko(const ConvParams& p, int nt, int ko, hipStream_t s) {
  if (!dma_x3_supported(p) || p.res || !p.relu || p.y_c8 || p.n_split > 1) return hipErrorInvalidValue;
#define DX3KO(N)                                       \
  switch (ko) {                                        \
    case 0: return dma_x3_ko_t<N, 0>(p, s);             \
    case 1: return dma_x3_ko_t<N, 1>(p, s);             \
    case 2: return dma_x3_ko_t<N, 2>(p, s);             \
    case 4: return dma_x3_ko_t<N, 4>(p, s);             \
    case 8: return dma_x3_ko_t<N, 8>(p, s);             \
    case 16: return dma_x3_ko_t<N, 16>(p, s);           \
    case 31: return dma_x3_ko_t<N, 31>(p, s);           \
    case 32: return dma_x3_ko_t<N, 32>(p, s);           \
    case 33: return dma_x3_ko_t<N, 33>(p, s);           \
    case 34: return dma_x3_ko_t<N, 34>(p, s);           \
    case 36: return dma_x3_ko_t<N, 36>(p, s);           \
    case 40: return dma_x3_ko_t<N, 40>(p, s);           \
    case 48: return dma_x3_ko_t<N, 48>(p, s);           \
  }
  if (nt == 5) DX3KO(5)
  if (nt == 8) DX3KO(8)
#undef DX3KO
  return hipErrorInvalidValue;
}
#endif

// bf16 image [npairs][3][cout_alloc][32] of an fp32 [cout_alloc][Kp] weight image (Kp % 16 == 0,
// npairs = ceil(Kp / 32)): piece pc of element (n, k) is the bf16 of w - (pieces < pc) (round to
// nearest, exact in double); element 8q + e of a 32-slot holds k = 32 pair + 4q + e (e < 4) or
// 32 pair + 16 + 4q + (e - 4) -- conv_dma_x3's operand order. Pair- and piece-major (round 5; was
// [cout_alloc][npairs][3][32]): the 16 rows one B-piece DMA instruction fetches are 1 KiB contiguous
// instead of 16 half-lines npairs * 192 B apart.
void dma_x3_weight_image(const float* w, int cout_alloc, int Kp, uint16_t* out) {
  const int npairs = (Kp / 16 + 1) / 2;
  for (int n = 0; n < cout_alloc; ++n)
    for (int pr = 0; pr < npairs; ++pr)
      for (int sl = 0; sl < 32; ++sl) {
        const int q = sl >> 3, e = sl & 7;
        const int k = 32 * pr + (e < 4 ? 4 * q + e : 16 + 4 * q + (e - 4));
        double r = k < Kp ? (double)w[(size_t)n * Kp + k] : 0.0;
        for (int pc = 0; pc < 3; ++pc) {
          float f = (float)r;
          uint32_t u;
          memcpy(&u, &f, 4);
          // round to nearest even on the upper 16 bits (finite weights)
          const uint16_t b = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
          const uint32_t ub = (uint32_t)b << 16;
          float fb;
          memcpy(&fb, &ub, 4);
          out[(((size_t)pr * 3 + pc) * cout_alloc + n) * 32 + sl] = b;
          r -= fb;
        }
      }
}

size_t dma_x3_weight_elems(int cout_alloc, int Kp) { return (size_t)cout_alloc * ((Kp / 16 + 1) / 2) * 96; }

// Tile choice: BM = 128 (mt = 2) and the widest N tile (16*NT, NT <= 9) dividing Cout.
// Measured (round 1, 30 clips of 32x112x112): BM = 128 beats 64 and 256 on every layer -- 256 halves
// occupancy (LDS + accumulators), 64 doubles the weight re-reads of the small-M layer4 convs -- and
// the widest N tile wins (the im2col A tile is read once); the ring depth (2, 3, 4 stages) changes
// layer1 by < 1 % (3: default; 4 loses a block per CU). force_nt > 0 restricts NT (A/B runs).
void conv_pick_tile(int M, int cout_p, int force_nt, int* mt_out, int* bn_out) {
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

// y = [relu](sum over splits, in split order, of part[split] + bias + res): fp32 channels-last,
// 4 floats per lane (Cout % 4 == 0)
__global__ __launch_bounds__(256) void split_sum_kernel(const float* __restrict__ part, int n_split, long n4, int co4,
                                                        const float* __restrict__ bias, const float* res, int relu,
                                                        float* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const f32x4* pp = reinterpret_cast<const f32x4*>(part);
  f32x4 v = pp[i];
  for (int k = 1; k < n_split; ++k) v += pp[(long)k * n4 + i];
  if (bias) v += reinterpret_cast<const f32x4*>(bias)[i % co4];
  if (res) v += reinterpret_cast<const f32x4*>(res)[i];
  if (relu)
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = relu1(v[c]);
  reinterpret_cast<f32x4*>(y)[i] = v;
}

hipError_t launch_split_sum(const ConvParams& p, hipStream_t s) {
  if (p.in_bf16 || p.out_bf16 || p.y_c8 || p.Cout % 4 || !p.part) return hipErrorInvalidValue;
  const long n4 = (long)p.M * p.Cout / 4;
  hipLaunchKernelGGL(split_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, p.part, p.n_split, n4,
                     p.Cout / 4, p.bias, (const float*)p.res, p.relu, (float*)p.y);
  return hipGetLastError();
}

// Split-K factor for conv_dma (fp32, channels-last output): as winot_split_for -- maps of <= 256
// output voxels per clip (layer4's temporal stride-2 conv at 112x112 clips: 184 tiles for 30 clips)
// split K into 4 ranges of >= 16 steps; the factor depends on the per-clip shape only, never on the
// batch size.
int dma_split_for(const ConvParams& p, int mt) {
  if (p.in_bf16 || p.out_bf16 || p.y_c8 || p.stem || mt != 2 || (p.vflags & CLASFV_VARIANT_NO_SPLIT_K)) return 1;
  if ((long)p.To * p.Ho * p.Wo > 256 || p.Kp / 16 < 4 * 16) return 1;
  return 4;
}

hipError_t launch_conv(const ConvParams& p, int mt, int bn, hipStream_t s) {
#ifdef CLASFV_KNOCKOUTS
  if (mt == 4 && p.in_bf16 && !p.stem) return launch_bf16_m4(p, bn, s);
#endif
  if (mt != 2) return hipErrorInvalidValue;
  if (p.stem) {  // fp32 input with 4 channels (3 + zero pad)
    if (bn == 48) return launch_stem<3>(p, s);
    if (bn == 64) return launch_stem<4>(p, s);
    return hipErrorInvalidValue;
  }
  return p.in_bf16 ? launch_typed<__bf16>(p, bn, s) : launch_typed<float>(p, bn, s);
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

bool stem_bf16_supported(const ConvParams& p) {
  return p.stem && p.out_bf16 && p.Cin == 4 && p.Cout == 64 && p.KT == 1 && p.KH == 7 && p.KW == 7 && p.st == 1 &&
         p.sh == 2 && p.sw == 2 && p.pt == 0 && p.ph == 3 && p.pw == 3 && p.relu && !p.res && p.bias &&
         p.To == p.Ti && (size_t)p.M < ((size_t)1 << 31);
}

bool stem_x3_supported(const ConvParams& p) {
  return !(p.vflags & CLASFV_VARIANT_NO_STEM_X3) && p.stem && !p.out_bf16 && !p.in_bf16 && p.Cin == 4 &&
         p.Cout == 48 && p.KT == 1 && p.KH == 7 && p.KW == 7 && p.st == 1 && p.sh == 2 && p.sw == 2 && p.pt == 0 &&
         p.ph == 3 && p.pw == 3 && !p.res && !p.x_c8 && p.To == p.Ti && (size_t)p.M < ((size_t)1 << 31);
}

// p.w: hi, mid, lo images, each [48][7 kh][8 kw][4 c] bf16 (engine.hip, clasfv_finalize).
hipError_t launch_stem_x3(const ConvParams& p, hipStream_t s) {
  if (!stem_x3_supported(p)) return hipErrorInvalidValue;
  // two blocks per CU (64.5 KiB of weight images each), or one item per block on small maps
  const int n_items = (int)((p.M + 255) / 256);
  const int grid = n_items >= 1024 ? 512 : (n_items + 7) / 8 * 8;
  hipLaunchKernelGGL(conv_stem_x3, dim3(grid), dim3(256), 0, s, p, n_items);
  return hipGetLastError();
}

// p.w: hi then lo image, each [64][7 kh][8 kw][4 c] bf16 (engine.hip, clasfv_finalize).
hipError_t launch_stem_bf16(const ConvParams& p, hipStream_t s) {
  if (!stem_bf16_supported(p)) return hipErrorInvalidValue;
  const int n_items = (int)((p.M + 255) / 256);
  const int grid = n_items >= 1024 ? 512 : (n_items + 7) / 8 * 8;
  hipLaunchKernelGGL(conv_stem_bf16, dim3(grid), dim3(256), 0, s, p, n_items);
  return hipGetLastError();
}

