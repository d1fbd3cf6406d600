// Fused full-resolution CLAS-FV decoder for gfx950 (fp32; bf16 MFMAs for comb_2 and the heads in
// bf16 engines: comb_2 on bf16 MFMAs).
//
// Reference (src/model/R2plus1D_18_MotionNet.py:39-71): five trilinear align_corners=True
// upsamplings of the encoder taps to (T,H,W), torch.cat to 1024 channels (1.64 GB at 32x112x112),
// conv 1x1x1 1024->64 + BN + ReLU, conv 64->64 + BN + ReLU, seg head 64->2, motion head 64->4 + tanh.
//
// Here: trilinear upsampling is linear and per channel, so comb_1(cat(up(f_i))) = sum_i up(W_i f_i).
// The 1x1x1 projections P_i = (s1*W_i) f_i are computed at tap resolution by the conv kernel
// (stem+layer1 share one resolution and are summed there), and this kernel, per output tile of one
// frame x 8 rows x 16 cols:
//   1. stages the rows x cols x 64-channel source windows of the four P tensors in LDS, already
//      blended in time (every voxel of a block shares its output frame, so the temporal lerp of
//      taps 1-3 is done once per staged pixel instead of once per voxel);
//   2. interpolates them bilinearly per voxel in registers (lane = voxel column, 16 channels per
//      lane) and adds b1 -> ReLU -> h1 (never written to HBM);
//   3. h2^T = W2 . h1^T on v_mfma_f32_16x16x4_f32: h1 is already the B operand in registers;
//   4. bias + ReLU, then heads^T = Wh . h2^T on MFMA again: the 16x16 accumulator layout of step 3
//      (rows = channels on lane groups, cols = voxels on lanes) is exactly the B-operand layout;
//   5. writes seg logits and tanh(motion) in the reference (N,C,T,H,W) layout, 64-B coalesced.
// 30 KB of LDS and <= 102 VGPRs per block: 5 blocks (5 waves per SIMD) per CU, so one block's
// staging latency hides behind the others' MFMAs (30 clips: 2.73 ms -> 1.69 ms with the shared W2
// loads, the blended staging and the occupancy).
#include "common.h"

#include <string.h>

namespace {

// floats per staged pixel: 64 channels + 8 pad. A ds_read_b128 lane group reads 8 distinct (source
// pixel px, channel group q) slots at 16-B quad (px * PIX / 4 + q) mod 16 = (2 px + q) mod 16: all
// distinct for the 2x-upsampled tap (PIX = 68 gave (px + q) mod 16, 2-way conflicts).
constexpr int PIX = 72;
constexpr int TILE_W = 16;
// Tile = TH rows x 16 columns of one frame, TH / 2 waves (2 voxel rows each). Source window bounds
// per tap (tap i: scale (in-1)/(out-1) < 2^-(i+1), so TH rows touch at most floor((TH-1) s) + 3
// source rows, 16 columns floor(15 s) + 3).
template <int TH>
struct DecGeo {
  static constexpr int NTHR = 32 * TH;
  static constexpr int rows(int i) { return ((TH - 1) >> (i + 1)) + 3; }
  static constexpr int cols(int i) { return (15 >> (i + 1)) + 3; }  // also the staging row pitch
  static constexpr int kMaxRows[4] = {rows(0), rows(1), rows(2), rows(3)};
  static constexpr int kMaxCols[4] = {cols(0), cols(1), cols(2), cols(3)};
  // tap 0 (stem + layer1) keeps the clip's frame rate: its temporal scale is exactly 1, one frame;
  // taps 1-3 read two frames and stage their temporal blend.
  static constexpr int kFrames[4] = {1, 2, 2, 2};
  static constexpr int kTapPix[4] = {rows(0) * cols(0), rows(1) * cols(1), rows(2) * cols(2), rows(3) * cols(3)};
  static constexpr int kPixOff[5] = {0, kTapPix[0], kTapPix[0] + kTapPix[1], kTapPix[0] + kTapPix[1] + kTapPix[2],
                                     kTapPix[0] + kTapPix[1] + kTapPix[2] + kTapPix[3]};
  static constexpr int STAGE_FLOATS = kPixOff[4] * PIX;
  // per-thread 16-byte staging elements per tap: ceil(rows * cols * 16 / NTHR), each kFrames loads
  static constexpr int ld(int i) { return (kTapPix[i] * 16 + NTHR - 1) / NTHR; }
  static constexpr int kLoads[4] = {ld(0), ld(1), ld(2), ld(3)};
  static constexpr int kLoadOff[4] = {0, ld(0), ld(0) + 2 * ld(1), ld(0) + 2 * ld(1) + 2 * ld(2)};
  static constexpr int kLoadsTotal = ld(0) + 2 * (ld(1) + ld(2) + ld(3));
  static constexpr int kLiveOff[5] = {0, ld(0), ld(0) + ld(1), ld(0) + ld(1) + ld(2), ld(0) + ld(1) + ld(2) + ld(3)};
};
// the 8 x 16 tile of rounds 1-4: 30 KB of staging, 5 blocks (4 in MODE 4) per CU
static_assert(DecGeo<8>::STAGE_FLOATS == 105 * PIX && DecGeo<8>::kLoadsTotal == 12, "8-row tile geometry");

struct Win {
  int t0, t1, r0, nr, c0, nc;
  float lt0, lt1;
};

__device__ inline void src_index(float s, int dst, int in, int& i0, int& i1, float& l0, float& l1) {
  const float f = s * (float)dst;
  i0 = min((int)floorf(f), in - 1);
  l1 = fminf(fmaxf(f - (float)i0, 0.f), 1.f);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l0 = 1.f - l1;
}

// The source-index table of one launch (DecParams::idx): per tap i at entry i (T + H + W), the T
// output frames' (t0, t1, lt0, lt1) -- the temporal blend the staging applies, already collapsed to
// one frame (t1 = t0, weights 1 and 0) where the decoder reads one (tap 0, or a zero second weight)
// -- then the H output rows' and the W output columns' src_index (i0, i1, l0, l1). The same device
// src_index over the same scales as the decoder's own evaluation, so the decoder reads back the
// values it used to compute per wave: ≈ 240 VALU of index arithmetic (floors, clamps, conversions)
// and ≈ 60 readfirstlanes per wave become a few scalar loads and one vector load per tap.
struct DecIdx {
  int i0, i1;
  float l0, l1;
};

__global__ __launch_bounds__(256) void decoder_index_kernel(DecParams p) {
  const int per = p.T + p.H + p.W;
  DecIdx* tab = reinterpret_cast<DecIdx*>(p.idx);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < 4 * per; e += gridDim.x * 256) {
    const int i = e / per, k = e - i * per;
    const DecTap& tp = p.tap[i];
    DecIdx d;
    if (k < p.T) {
      float la, lb;
      src_index(tp.st, k, tp.T, d.i0, d.i1, la, lb);
      const bool two = lb > 0.f && d.i1 != d.i0 && i > 0;  // decoder_kernel: DecGeo::kFrames[i] == 2
      d.i1 = two ? d.i1 : d.i0;
      d.l0 = two ? la : 1.f;
      d.l1 = two ? lb : 0.f;
    } else if (k < p.T + p.H) {
      src_index(tp.sh, k - p.T, tp.H, d.i0, d.i1, d.l0, d.l1);
    } else {
      src_index(tp.sw, k - p.T - p.H, tp.W, d.i0, d.i1, d.l0, d.l1);
    }
    tab[e] = d;
  }
}

// tanh(x) = 1 - 2 / (e^(2x) + 1) on v_exp_f32 and v_rcp_f32: a few VALU instructions instead of
// tanhf's ~30 (the decoder is VALU-issue bound); absolute error ~1e-7, saturates to +-1 exactly
__device__ inline float fast_tanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f); }

// block- / wave-uniform values computed on the VALU, moved to SGPRs: the address arithmetic and the
// branches that use them become scalar
__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

__device__ inline int xcd_swizzle_d(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// single-lane f32 FMA / multiply kept as one v_fma_f32 / v_mul_f32: on f32x4 values the compiler emits
// v_pk_fma_f32 / v_pk_mul_f32, which beside other waves' MFMAs cost more issue than two scalar ops
// (MI355X_MICROARCH.md, "packed f32 VALU: an anti-lever beside MFMAs")
__device__ inline float fma1(float a, float b, float c) {
  float d;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ inline float mul1(float a, float b) {
  float d;
  asm("v_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

__device__ inline bf16x8 to_bf16x8(f32x4 a, f32x4 b) {
  return bf16x8{(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3],
                (__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
}

// x = hi + lo with hi = bf16(x), lo = bf16(x - hi): the pair carries ~16 mantissa bits
__device__ inline void split_bf16x8(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& lo) {
  hi = to_bf16x8(a, b);
  f32x4 ra, rb;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ra[e] = a[e] - (float)hi[e];
    rb[e] = b[e] - (float)hi[4 + e];
  }
  lo = to_bf16x8(ra, rb);
}

// x = hi + mid + lo, each a bf16 of the remainder (round to nearest): 24 mantissa bits, fp32's
__device__ inline void split3_bf16x8(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
  hi = to_bf16x8(a, b);
  f32x4 ra, rb;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ra[e] = a[e] - (float)hi[e];
    rb[e] = b[e] - (float)hi[4 + e];
  }
  mid = to_bf16x8(ra, rb);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ra[e] -= (float)mid[e];
    rb[e] -= (float)mid[4 + e];
  }
  lo = to_bf16x8(ra, rb);
}

// Steps 3-5 of the bf16-engine decoder (see decoder_kernel): h1[mt][c][j] = channel 16c + 4q + j of
// voxel (row h0 + 2 wid + mt, column w0 + l16). comb_2 runs as three bf16 products per K block
// (hi.hi + hi.lo + lo.hi of the split operands: ~fp32 accuracy at 6 instead of 32 MFMA slots).
// X3 (fp32 engines): comb_2 as six bf16 products of 3-way split operands (lo.hi + hi.lo + mid.mid +
// mid.hi + hi.mid + hi.hi, smallest first; the dropped terms are below 2^-24 of the product) with fp32
// accumulation -- fp32-accurate, on the bf16 matrix rate (12 instead of 32 MFMA slots; on gfx950 the
// f32 MFMA shares the f32 vector rate with the interpolation, which the bf16 MFMA does not). W2's
// pieces come split on the host (DecParams::w2x3), h1's are split here.
// W2S (bf16 engines, the knock-out builds' legacy form): W2's hi / lo pieces split here from the fp32
// W2 in every wave; otherwise read from DecParams::w2x3, whose mid piece is exactly that lo (the
// bf16 of the remainder w - hi, exact in fp32, rounded to nearest either way): bit-identical, 64 split
// values per lane fewer
template <bool X3, bool HX3, bool W2S = false>
__device__ inline void decoder_heads_bf16(const DecParams& p, const f32x4 (&h1)[2][4], int t, int n, int h0, int w0,
                                          int wid, int q, int l16) {
  bf16x8 hh[2][2], hl[2][2], hm[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if constexpr (X3)
        split3_bf16x8(h1[mt][2 * kb], h1[mt][2 * kb + 1], hh[mt][kb], hm[mt][kb], hl[mt][kb]);
      else
        split_bf16x8(h1[mt][2 * kb], h1[mt][2 * kb + 1], hh[mt][kb], hl[mt][kb]);
    }
  f32x4 acc[2][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    [[maybe_unused]] const float* wr = p.w2 + (16 * nt + l16) * 64 + 4 * q;
    bf16x8 wh_[2], wl_[2], wm_[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8* w3 = reinterpret_cast<const bf16x8*>(p.w2x3) + ((nt * 2 + kb) * 16 + l16) * 4 + q;
      if constexpr (X3) {
        wh_[kb] = w3[0];
        wm_[kb] = w3[512];
        wl_[kb] = w3[1024];
      } else if constexpr (!W2S) {
        wh_[kb] = w3[0];
        wl_[kb] = w3[512];
      } else {
        split_bf16x8(*reinterpret_cast<const f32x4*>(wr + 32 * kb), *reinterpret_cast<const f32x4*>(wr + 32 * kb + 16),
                     wh_[kb], wl_[kb]);
      }
    }
    const f32x4 bb = *reinterpret_cast<const f32x4*>(p.b2 + 16 * nt + 4 * q);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 a = bb;  // the bias rides in the accumulator
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl_[kb], hh[mt][kb], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_[kb], hl[mt][kb], a, 0, 0, 0);
        if constexpr (X3) {
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm_[kb], hm[mt][kb], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm_[kb], hh[mt][kb], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_[kb], hm[mt][kb], a, 0, 0, 0);
        }
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_[kb], hh[mt][kb], a, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = relu1(a[r]);
      acc[mt][nt] = a;  // h2^T[ch = 16nt + 4q + r][voxel l16]
    }
  }
  f32x4 hb;
#pragma unroll
  for (int r = 0; r < 4; ++r) hb[r] = 4 * q + r < 6 ? p.bh[4 * q + r] : 0.f;
  const size_t HW = (size_t)p.H * p.W;
  const size_t TH = (size_t)p.T * HW;
  f32x4 outs[2] = {hb, hb};  // head bias (rows 4q + r < 6) in the accumulator
  if constexpr (HX3) {
    // heads^T = Wh . h2^T as six split-bf16 products too: a lane's accumulators hold channels
    // 16nt + 4q + r, i.e. K block kb = {nt 2kb, 2kb + 1} in the comb_2 operand order; Wh's pieces
    // (16 rows, 6 used) come split on the host behind W2's (fp32-accurate; the f32 MFMAs they replace
    // shared the f32 rate with the interpolation)
    const bf16x8* h3 = reinterpret_cast<const bf16x8*>(p.w2x3) + 3 * 4096 / 8 + l16 * 4 + q;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 wh_ = h3[kb * 64], wm_ = h3[128 + kb * 64], wl_ = h3[256 + kb * 64];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        bf16x8 vh, vm, vl;
        split3_bf16x8(acc[mt][2 * kb], acc[mt][2 * kb + 1], vh, vm, vl);
        f32x4 o = outs[mt];
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl_, vh, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_, vl, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm_, vm, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm_, vh, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_, vm, o, 0, 0, 0);
        outs[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh_, vh, o, 0, 0, 0);
      }
    }
  } else {
    // heads in fp32 (they produce the logits whose sign is the mask): heads^T = Wh . h2^T on
    // v_mfma_f32_16x16x4_f32, the accumulator layout being the B operand layout (k = 16nt + 4q + r)
    f32x4 wh[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      wh[nt] = *reinterpret_cast<const f32x4*>(p.wh + (l16 & 7) * 64 + 16 * nt + 4 * q);
      if (l16 >= 8) wh[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          outs[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wh[nt][r], acc[mt][nt][r], outs[mt], 0, 0, 0);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int hr = h0 + 2 * wid + mt;
    const f32x4 out = outs[mt];
    if (q < 2) {
      const size_t pix = (size_t)t * HW + (size_t)hr * p.W + (w0 + l16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 4 * q + r;
        if (co >= 6) continue;
        const float v = out[r];
        if (co < 2)
          p.seg[((size_t)n * 2 + co) * TH + pix] = v;
        else
          p.mot[((size_t)n * 4 + (co - 2)) * TH + pix] = fast_tanh(v);
      }
    }
  }
}

// (Heads as VALU dot products + a 4-lane-group reduction instead of the 16-row head MFMA of which 6
// rows are used measured slower: 1.83 vs 1.70 ms per 30 clips -- the interpolation already loads VALU.)
// BF = 1 (BASELINE config[4]): comb_2 on v_mfma_f32_16x16x32_bf16 with split (hi + lo) bf16 h1 and W2
// (one 32-deep K block = the 8 channels 16c + 4q + j, c in {2kb, 2kb+1}, that lane group q already
// holds, so both operands keep the fp32 path's register layout), fp32 accumulation; fp32 heads.
// MODE: 0 = fp32 (v_mfma_f32_16x16x4_f32 comb_2), 1 = bf16 comb_2, 4 = fp32-accurate comb_2 on six
// split-bf16 products (the fp32 engines' default); timing knock-outs for tools/convbench.hip
// (CLASFV_KNOCKOUTS builds only; wrong results): 2 = no comb_2 / head MFMAs, 3 = no interpolation.
// TROWS: tile rows (8: 4 waves per block; 16: 8 waves, half the blocks and less halo per voxel)
// MODE + 8 (SC): the staging blend and the interpolation as single-lane v_fma_f32 / v_mul_f32
// (the same operations and order as the packed form, so bit-identical)
// MODE_ + 16 (LIX, knock-out builds): every wave evaluates its source indices itself (src_index per
// tap and voxel row / column, the staging windows) instead of reading DecParams::idx; + 32 (bf16
// engines): W2's pieces split in the kernel (decoder_heads_bf16's W2S). Both bit-identical. + 64
// (knock-out builds): the fp32 engines' form at five waves per SIMD (96 VGPRs, a few spilled).
template <int MODE_, int TROWS = 8>
__global__ __launch_bounds__(32 * TROWS) __attribute__((amdgpu_waves_per_eu(((MODE_ & 7) == 4 && !(MODE_ & 64)) ? 4 : 5, ((MODE_ & 7) == 4 && !(MODE_ & 64)) ? 4 : 5))) void decoder_kernel(DecParams p) {
  constexpr int MODE = MODE_ & 7;
  constexpr bool SC = (MODE_ & 8) != 0;
  constexpr bool LIX = (MODE_ & 16) != 0;
  constexpr bool W2S = (MODE_ & 32) != 0;
  using G = DecGeo<TROWS>;
  constexpr int TILE_H = TROWS, NTHR = G::NTHR;
  constexpr int BF = MODE == 1 || MODE == 4;
  extern __shared__ __align__(16) float smem[];
  float* stage = smem;  // G::STAGE_FLOATS

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // voxel-row loops below are scalar branches
  const int q = lane >> 4, l16 = lane & 15;
  const int tiles_w = p.W / TILE_W, tiles = (p.H / TILE_H) * tiles_w;
  // 1-D grid, XCD-aware: consecutive logical tiles (row-major in a frame, then frame, then clip) land
  // on one XCD, so the halo rows / columns and the temporal source frames that neighbouring tiles
  // share are served by that XCD's L2 instead of being fetched again by another XCD
  int lt = xcd_swizzle_d(blockIdx.x, gridDim.x);
  const int tile = lt % tiles;
  lt /= tiles;
  const int t = lt % p.T, n = lt / p.T;
  const int h0 = (tile / tiles_w) * TILE_H, w0 = (tile % tiles_w) * TILE_W;


  // Source windows of the four taps: the tile's rows h0 .. h0 + TILE_H - 1 read source rows
  // i0(h0) .. i1(h0 + TILE_H - 1) (i1 = min(floor + 1, in - 1), the window's last row), columns the same
  const DecIdx* tab = reinterpret_cast<const DecIdx*>(p.idx);
  const int per = p.T + p.H + p.W;
  Win win[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const DecTap& tp = p.tap[i];
    Win w;
    if constexpr (LIX) {
      int a, b;
      float la, lb;
      src_index(tp.st, t, tp.T, a, b, la, lb);
      const bool two = lb > 0.f && b != a && G::kFrames[i] == 2;  // else the blend below is exactly P[t0]
      w.t0 = uni(a);
      w.t1 = uni(two ? b : a);
      w.lt0 = unif(two ? la : 1.f);
      w.lt1 = unif(two ? lb : 0.f);
      const int r0 = min((int)floorf(tp.sh * (float)h0), tp.H - 1);
      const int r1 = min((int)floorf(tp.sh * (float)(h0 + TILE_H - 1)) + 1, tp.H - 1);
      const int c0 = min((int)floorf(tp.sw * (float)w0), tp.W - 1);
      const int c1 = min((int)floorf(tp.sw * (float)(w0 + TILE_W - 1)) + 1, tp.W - 1);
      w.r0 = uni(r0);
      w.nr = uni(min(r1 - r0 + 1, G::kMaxRows[i]));
      w.c0 = uni(c0);
      w.nc = uni(min(c1 - c0 + 1, G::kMaxCols[i]));
    } else {
      const DecIdx* ti = tab + i * per;
      const DecIdx ft = ti[t];  // block-uniform: scalar loads
      w.t0 = ft.i0;
      w.t1 = ft.i1;
      w.lt0 = ft.l0;
      w.lt1 = ft.l1;
      const int r0 = ti[p.T + h0].i0, r1 = ti[p.T + h0 + TILE_H - 1].i1;
      const int c0 = ti[per - p.W + w0].i0, c1 = ti[per - p.W + w0 + TILE_W - 1].i1;
      w.r0 = r0;
      w.nr = min(r1 - r0 + 1, G::kMaxRows[i]);
      w.c0 = c0;
      w.nc = min(c1 - c0 + 1, G::kMaxCols[i]);
    }
    win[i] = w;
  }
  // All staging loads are issued before the first LDS write (fixed per-tap trip counts, predicated),
  // so one block waits for one HBM/L2 latency instead of one per 16-byte chunk.
  f32x4 buf[G::kLoadsTotal];
  bool live[G::kLiveOff[4]];  // per (tap, k): the staged element exists in the window
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const DecTap& tp = p.tap[i];
    const Win& w = win[i];
    // staged with the constant row pitch G::kMaxCols[i] (the decode is a division by a constant;
    // columns past the window's nc are not loaded and never read)
    // 32-bit element offsets (the launcher checks every tap tensor stays below 2^31 floats): the
    // window origin of each source frame is scalar, the per-lane part one multiply per element
    const int base0 = (((n * tp.T + w.t0) * tp.H + w.r0) * tp.W + w.c0) * 64;
    const int base1 = base0 + (w.t1 - w.t0) * tp.H * tp.W * 64;
#pragma unroll
    for (int k = 0; k < G::kLoads[i]; ++k) {
      const int e = tid + NTHR * k;
      const int c4 = e & 15, px = e >> 4;
      const int rr = px / G::kMaxCols[i], cc = px - rr * G::kMaxCols[i];
      const bool lv = e < G::kTapPix[i] * 16 && rr < w.nr && cc < w.nc;
      live[G::kLiveOff[i] + k] = lv;
      const int lo = (rr * tp.W + cc) * 64 + c4 * 4;
#pragma unroll
      for (int f = 0; f < G::kFrames[i]; ++f) {
        f32x4& v = buf[G::kLoadOff[i] + k * G::kFrames[i] + f];
        if (lv) v = *reinterpret_cast<const f32x4*>(tp.p + (f ? base1 : base0) + lo);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const Win& w = win[i];
    float* dst = stage + G::kPixOff[i] * PIX;
#pragma unroll
    for (int k = 0; k < G::kLoads[i]; ++k) {
      const int e = tid + NTHR * k;
      if (live[G::kLiveOff[i] + k]) {
        f32x4 v = buf[G::kLoadOff[i] + k * G::kFrames[i]];
        if (G::kFrames[i] == 2) {
          const f32x4 v1 = buf[G::kLoadOff[i] + k * G::kFrames[i] + 1];
          if constexpr (SC) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fma1(v[e], w.lt0, mul1(v1[e], w.lt1));
          } else {
            v = v * w.lt0 + v1 * w.lt1;
          }
        }
        *reinterpret_cast<f32x4*>(dst + (e >> 4) * PIX + (e & 15) * 4) = v;
      }
    }
  }
  __syncthreads();

  // ---- per voxel row (mt): 2. interpolate, 3. comb_2 on MFMA, 4. heads on MFMA, 5. store.
  // lane = (voxel column l16, channel group q): h1[c][j] holds channel 16c + 4q + j.
  const size_t HW = (size_t)p.H * p.W;
  const size_t TH = (size_t)p.T * HW;
  // Both voxel rows of the wave are interpolated first, then share every W2 fragment load (W2 is
  // re-read from L1/L2 once per wave rather than once per row: the loads were the kernel's fixed cost).
  // Separable form, W then H (PyTorch's nesting): the wave's two voxel rows hr, hr + 1 (every tap
  // upsamples by more than 2, so they touch at most 3 consecutive source rows, wave-uniformly) share
  // each source row's column interpolation hx = lx0 P[r][x0] + lx1 P[r][x1]: 8 LDS reads per source
  // row, 16-24 per tap for both rows instead of 32.
  f32x4 h1[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int c = 0; c < 4; ++c) h1[mt][c] = *reinterpret_cast<const f32x4*>(p.b1 + 16 * c + 4 * q);
  const int hr = h0 + 2 * wid;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (MODE == 3) {  // knock-out: one LDS read per channel group instead of the interpolation
#pragma unroll
      for (int c = 0; c < 4; ++c) h1[0][c] += *reinterpret_cast<const f32x4*>(stage + G::kPixOff[i] * PIX + 4 * q + 16 * c + l16 * PIX);
      continue;
    }
    const DecTap& tp = p.tap[i];
    const Win& w = win[i];
    int x0, x1, ya0, ya1, yb0, yb1;
    float lx0, lx1, la0, la1, lb0, lb1;
    if constexpr (LIX) {
      src_index(tp.sw, w0 + l16, tp.W, x0, x1, lx0, lx1);
      src_index(tp.sh, hr, tp.H, ya0, ya1, la0, la1);
      src_index(tp.sh, hr + 1, tp.H, yb0, yb1, lb0, lb1);
      ya0 = uni(ya0), ya1 = uni(ya1), yb0 = uni(yb0), yb1 = uni(yb1);
      la0 = unif(la0), la1 = unif(la1), lb0 = unif(lb0), lb1 = unif(lb1);
    } else {
      const DecIdx* ti = tab + i * per;
      const DecIdx cx = ti[per - p.W + w0 + l16];  // one 16-B load per lane
      const DecIdx ra = ti[p.T + hr], rb = ti[p.T + hr + 1];  // wave-uniform: scalar loads
      x0 = cx.i0, x1 = cx.i1, lx0 = cx.l0, lx1 = cx.l1;
      ya0 = ra.i0, ya1 = ra.i1, la0 = ra.l0, la1 = ra.l1;
      yb0 = rb.i0, yb1 = rb.i1, lb0 = rb.l0, lb1 = rb.l1;
    }
    const int nrows = yb1 - ya0 + 1;  // 1..3, wave-uniform
    const float* fb = stage + G::kPixOff[i] * PIX + 4 * q + (ya0 - w.r0) * G::kMaxCols[i] * PIX;
    const float* c0p = fb + (x0 - w.c0) * PIX;
    const float* c1p = fb + (x1 - w.c0) * PIX;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k >= nrows) break;
      // weights of source row ya0 + k in output rows hr (wa) and hr + 1 (wb)
      // source row ya0 + k feeds output row hr (ta) / hr + 1 (tb); a row that feeds only one of them
      // (the outer rows when nrows = 3) skips the other's update, whose weight is exactly 0 (scalar
      // branches: every condition is wave-uniform)
      const bool ta = k == 0 || ya1 - ya0 == k, tb = yb0 - ya0 == k || yb1 - ya0 == k;
      const float wa = (k == 0 ? la0 : 0.f) + (ya1 - ya0 == k ? la1 : 0.f);
      const float wb = (yb0 - ya0 == k ? lb0 : 0.f) + (yb1 - ya0 == k ? lb1 : 0.f);
      const int ro = k * G::kMaxCols[i] * PIX;
      f32x4 hx[4];
      if constexpr (SC) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(c0p + ro + 16 * c), a1 = *reinterpret_cast<const f32x4*>(c1p + ro + 16 * c);
#pragma unroll
          for (int e = 0; e < 4; ++e) hx[c][e] = fma1(a0[e], lx0, mul1(a1[e], lx1));
        }
        if (ta) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) h1[0][c][e] = fma1(hx[c][e], wa, h1[0][c][e]);
        }
        if (tb) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) h1[1][c][e] = fma1(hx[c][e], wb, h1[1][c][e]);
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          hx[c] = *reinterpret_cast<const f32x4*>(c0p + ro + 16 * c) * lx0 +
                  *reinterpret_cast<const f32x4*>(c1p + ro + 16 * c) * lx1;
        if (ta) {
#pragma unroll
          for (int c = 0; c < 4; ++c) h1[0][c] += hx[c] * wa;
        }
        if (tb) {
#pragma unroll
          for (int c = 0; c < 4; ++c) h1[1][c] += hx[c] * wb;
        }
      }
      // one source row's 8 LDS reads in flight at a time (hoisting more spills)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) h1[mt][c][j] = relu1(h1[mt][c][j]);

  if constexpr (BF) {
    decoder_heads_bf16<MODE == 4, true, W2S>(p, h1, t, n, h0, w0, wid, q, l16);
    return;
  }
  // 3. h2^T[n][v] = sum_k W2[n][k] h1[v][k]; MFMA j of lane group q covers k = 16c + 4q + j
  // (W2 rows of the next 16-channel tile are prefetched while the current one runs on MFMA)
  f32x4 acc[2][4], wa[4], wn[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wa[c] = *reinterpret_cast<const f32x4*>(p.w2 + l16 * 64 + 16 * c + 4 * q);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    if (nt < 3) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        wn[c] = *reinterpret_cast<const f32x4*>(p.w2 + ((nt + 1) * 16 + l16) * 64 + 16 * c + 4 * q);
    }
    const f32x4 bb = *reinterpret_cast<const f32x4*>(p.b2 + 16 * nt + 4 * q);
    acc[0][nt] = bb;  // the bias rides in the accumulator
    acc[1][nt] = bb;
    if constexpr (MODE == 2) {  // knock-out: no MFMA
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt][nt] += wa[nt] * h1[mt][nt];
    } else {
      // one accumulator chain at a time (alternating the two rows' chains measured the same: 1.608 vs
      // 1.598 ms, profiles/r03d_decoder_variants.txt)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[c][j], h1[mt][c][j], acc[mt][nt], 0, 0, 0);
    }
    // acc[mt][nt][r] = h2^T[ch = 16nt + 4q + r][voxel l16]
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mt][nt][r] = relu1(acc[mt][nt][r]);
#pragma unroll
    for (int c = 0; c < 4; ++c) wa[c] = wn[c];
  }
  // 4. heads^T[co][v] = sum_k Wh[co][k] h2^T[k][v]; the accumulator layout is the B operand
  f32x4 wh[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    wh[nt] = *reinterpret_cast<const f32x4*>(p.wh + (l16 & 7) * 64 + 16 * nt + 4 * q);
    if (l16 >= 8) wh[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 hb;
#pragma unroll
  for (int r = 0; r < 4; ++r) hb[r] = 4 * q + r < 6 ? p.bh[4 * q + r] : 0.f;
  f32x4 outs[2] = {hb, hb};  // head bias (rows 4q + r < 6) in the accumulator
  if constexpr (MODE == 2) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) outs[mt] += wh[nt] * acc[mt][nt];
  } else {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          outs[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wh[nt][r], acc[mt][nt][r], outs[mt], 0, 0, 0);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int hr = h0 + 2 * wid + mt;
    const f32x4 out = outs[mt];
    // 5. out[r] = head (4q + r) at voxel (hr, w0 + l16)
    if (q < 2) {
      const size_t pix = (size_t)t * HW + (size_t)hr * p.W + (w0 + l16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 4 * q + r;
        if (co >= 6) continue;
        const float v = out[r];
        if (co < 2)
          p.seg[((size_t)n * 2 + co) * TH + pix] = v;
        else
          p.mot[((size_t)n * 4 + (co - 2)) * TH + pix] = fast_tanh(v);
      }
    }
  }
}

}  // namespace

static hipError_t launch_dec(const DecParams& p, hipStream_t s, int mode, int th = 8) {
  if (p.tap[0].T != p.T) return hipErrorInvalidValue;  // tap 0 is staged as a single frame
  for (int i = 0; i < 4; ++i)  // the staging loads use 32-bit element offsets
    if ((size_t)p.N * p.tap[i].T * p.tap[i].H * p.tap[i].W * 64 >= ((size_t)1 << 31)) return hipErrorInvalidValue;
  if (p.H % th || p.W % TILE_W) return hipErrorInvalidValue;
  const size_t nb = (size_t)(p.H / th) * (p.W / TILE_W) * p.T * p.N;
  if (nb >= ((size_t)1 << 31)) return hipErrorInvalidValue;
  static_assert(DecGeo<16>::STAGE_FLOATS * 4 <= 64 * 1024, "default dynamic LDS limit");
  const size_t lds = (size_t)(th == 16 ? DecGeo<16>::STAGE_FLOATS : DecGeo<8>::STAGE_FLOATS) * 4;
  void (*k)(DecParams) = nullptr;
  if (th == 8) k = mode == 1 ? decoder_kernel<1> : mode == 4 ? decoder_kernel<4> : mode == 0 ? decoder_kernel<0> : nullptr;
#ifdef CLASFV_KNOCKOUTS
  if (th == 16 && mode < 16) k = mode == 1 ? decoder_kernel<1, 16> : mode == 4 ? decoder_kernel<4, 16> : decoder_kernel<0, 16>;
  if (mode == 2) k = th == 16 ? decoder_kernel<2, 16> : decoder_kernel<2>;
  if (mode == 3) k = th == 16 ? decoder_kernel<3, 16> : decoder_kernel<3>;
  if (mode == 12) k = th == 16 ? decoder_kernel<12, 16> : decoder_kernel<12>;
  if (mode == 9) k = th == 16 ? decoder_kernel<9, 16> : decoder_kernel<9>;
  // the round-6 forms before the index table and the host-split bf16 W2 pieces
  if (th == 8 && mode == 1 + 16 + 32) k = decoder_kernel<1 + 16 + 32>;
  if (th == 8 && mode == 4 + 16) k = decoder_kernel<4 + 16>;
  if (th == 8 && mode == 0 + 16) k = decoder_kernel<0 + 16>;
  if (th == 8 && mode == 1 + 16) k = decoder_kernel<1 + 16>;
  if (th == 8 && mode == 1 + 32) k = decoder_kernel<1 + 32>;
  if (th == 8 && mode == 4 + 64) k = decoder_kernel<4 + 64>;
#endif
  if (!k) return hipErrorInvalidValue;
  if (!(mode & 16)) {  // the source-index table this launch reads, filled on the same stream first
    if (!p.idx) return hipErrorInvalidValue;
    const int ne = 4 * (p.T + p.H + p.W);
    hipLaunchKernelGGL(decoder_index_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, s, p);
  }
  hipLaunchKernelGGL(k, dim3((unsigned)nb), dim3(32 * th), lds, s, p);
  return hipGetLastError();
}

// DecParams::w2x3 of the X3 decoder: W2 (64 x 64, [n][k]) then Wh (8 x 64, rows 6, 7 zero; padded
// to the 16 MFMA rows) as hi, mid and lo bf16 pieces (each the bf16, round to nearest, of the
// remainder in double) in the lanes' operand order: W2 [piece][nt][kb][l16][q][e] at 0, Wh
// [piece][kb][l16][q][e] at 3 * 4096; element e of lane (l16, q) is column 32 kb + 4q + (e < 4 ? e :
// 12 + e) of row 16 nt + l16 (Wh: row l16).
void decoder_x3_weights(const float* w2, const float* wh, uint16_t* out) {
  auto put = [&](double r, size_t i0, size_t stride) {
    for (int pc = 0; pc < 3; ++pc) {
      float f = (float)r;
      uint32_t u;
      memcpy(&u, &f, 4);
      const uint16_t b = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
      const uint32_t ub = (uint32_t)b << 16;
      float fb;
      memcpy(&fb, &ub, 4);
      out[i0 + pc * stride] = b;
      r -= fb;
    }
  };
  for (int nt = 0; nt < 4; ++nt)
    for (int kb = 0; kb < 2; ++kb)
      for (int l = 0; l < 16; ++l)
        for (int q = 0; q < 4; ++q)
          for (int e = 0; e < 8; ++e)
            put(w2[(16 * nt + l) * 64 + 32 * kb + 4 * q + (e < 4 ? e : 12 + e)],
                ((((size_t)nt * 2 + kb) * 16 + l) * 4 + q) * 8 + e, 4096);
  for (int kb = 0; kb < 2; ++kb)
    for (int l = 0; l < 16; ++l)
      for (int q = 0; q < 4; ++q)
        for (int e = 0; e < 8; ++e)
          put(l < 8 ? wh[l * 64 + 32 * kb + 4 * q + (e < 4 ? e : 12 + e)] : 0.0,
              3 * 4096 + (((size_t)kb * 16 + l) * 4 + q) * 8 + e, 1024);
}

// 8-row tiles. 16-row tiles (convbench ko + 16 only) are bit-identical; convbench 1.293 -> 1.256 ms per
// 30 clips on cold taps (profiles/r05n_decoder_16row_tiles.txt), but 1.275-1.280 -> 1.289-1.294 in the
// forward, whose taps were just written (profiles/r05p_decoder_rows_forward_ab.txt). (MODE 1 at 16 rows:
// 1.176 -> 1.281 ms, a 512-thread block at 5 waves per SIMD leaves 4 resident.)
hipError_t launch_decoder(const DecParams& p, hipStream_t s) {
  if ((p.x3 || p.bf16) && !p.w2x3) return hipErrorInvalidValue;  // the split-bf16 heads' Wh pieces
  const int mode = p.bf16 ? 1 : p.x3 ? 4 : 0;
  return launch_dec(p, s, mode, 8);
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: ko 0 = 8-row tiles; 2, 3 = decoder_kernel's knock-out modes; + 16: 16-row tiles;
// + 32: single-lane interpolation FMAs; + 64: per-wave index arithmetic (no table); + 128: bf16 W2
// split in the kernel; + 256: the fp32 engines' decoder at five waves per SIMD
hipError_t launch_decoder_ko(const DecParams& p, hipStream_t s, int ko) {
  const int m = ko & 15;
  const int base = m == 2 || m == 3 ? m : (p.bf16 ? 1 : p.x3 ? 4 : 0);
  int mode = (ko & 32) && (base == 1 || base == 4) ? base + 8 : base;
  if (ko & 64) mode += 16;
  if ((ko & 128) && base == 1) mode += 32;
  if ((ko & 256) && base == 4) mode += 64;
  return launch_dec(p, s, mode, (ko & 16) ? 16 : 8);
}
#endif
