// Memory-bound per-video kernels of the CLAS-FV clip pipeline (gfx950).
//
//   build_clips        divide_to_consecutive_clips        src/fuse_utils.py:16-33
//   pass_labels        softmax -> temporal resample -> argmax   src/fuse_utils.py:53-80
//   logit_margin       l1 - l0 per clip voxel (the multi-GPU exchange payload)
//   fuse_votes         per-frame label fusion            src/fuse_utils.py:82-100
//   warp               generate_2dmotion_field + grid_sample   src/transform_utils.py:14-34
//   warp_backward      its gradients (autograd of the training losses, src/clasfv_losses.py:29-136)
//   zeroone_normalize  zeroone_normalizer                src/echonet_dataset.py:38-50
//   preprocess_video   frames -> (3,T,H,W) + trilinear resize   motion_segment.py:96-106
//
// Interpolation arithmetic follows PyTorch's CPU upsample kernel bit for bit (checked against
// F.interpolate in tests): scale = (float)in/out, src = fma(scale, dst + 0.5, -0.5) clamped at 0,
// value = fma(x[i0], l0, x[i1] * l1).
#include <float.h>
#include <stdlib.h>

#include "common.h"

#include "clasfv.h"
#include "plumbing.h"

// Every fused multiply-add below is written out (fmaf) where PyTorch's CPU kernels contract one;
// nothing else may be contracted (HIP's __fmul_rn etc. are plain operators defined in a header this pragma does not reach, so
// the operators are written out here).
#pragma clang fp contract(off)

namespace {

__device__ inline int round_half_even_div32(int t) {
  const int q = t >> 5, r = t & 31;
  if (r > 16) return q + 1;
  if (r < 16) return q;
  return q + (q & 1);
}

struct Lin {
  int i0, i1;
  float l0, l1;
};

// align_corners=False source index for output index dst of a t_in -> t_out resampling.
__device__ inline Lin lin_ac_false(int t_in, int t_out, int dst) {
  Lin r;
  const float scale = (float)t_in / (float)t_out;
  float src = fmaf(scale, (float)dst + 0.5f, -0.5f);
  src = fmaxf(src, 0.f);
  r.i0 = min((int)floorf(src), t_in - 1);
  r.l1 = fminf(fmaxf(src - (float)r.i0, 0.f), 1.f);
  r.i1 = r.i0 + (r.i0 < t_in - 1 ? 1 : 0);
  r.l0 = 1.f - r.l1;
  return r;
}

__device__ inline float lerp_t(float a, float b, float l0, float l1) { return fmaf(a, l0, (b * l1)); }

// ---- build_clips ------------------------------------------------------------------------------
__global__ void build_clips_kernel(const float* __restrict__ video, int T, int HW, const int32_t* __restrict__ table,
                                   int interp, float* __restrict__ clips) {
  const int clip = blockIdx.z, fr = blockIdx.y;  // fr in [0, 3*32)
  const int c = fr >> 5, f = fr & 31;
  const int shift = table[2 * clip], j0 = table[2 * clip + 1];
  const int tk = T - shift;
  const int tf = j0 + f;  // frame index in the (resampled) shifted video
  const int tc = 32 * round_half_even_div32(tk);
  const float* vc = video + (size_t)c * T * HW;
  float* out = clips + (((size_t)clip * 3 + c) * 32 + f) * HW;
  const bool resample = interp && (tk & 31) && tk != tc;
  Lin L = {0, 0, 1.f, 0.f};
  if (resample) L = lin_ac_false(tk, tc, tf);
  const float* a = vc + (size_t)(shift + (resample ? L.i0 : tf)) * HW;
  const float* b = vc + (size_t)(shift + (resample ? L.i1 : tf)) * HW;
  if ((HW & 3) == 0 && (((uintptr_t)video | (uintptr_t)clips) & 15) == 0) {  // 16-B vectors, the same per-element arithmetic
    const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
    const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
    f32x4* o4 = reinterpret_cast<f32x4*>(out);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (HW >> 2); i += gridDim.x * blockDim.x) {
      f32x4 v = a4[i];
      if (resample) {
        const f32x4 w = b4[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = lerp_t(v[e], w[e], L.l0, L.l1);
      }
      o4[i] = v;
    }
    return;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x)
    out[i] = resample ? lerp_t(a[i], b[i], L.l0, L.l1) : a[i];
}

// ---- pass_labels ------------------------------------------------------------------------------
struct PassTable {
  int clip0[CLASFV_MAX_PASSES];
};

__device__ inline void softmax2(float x0, float x1, float& p0, float& p1) {
  const float m = fmaxf(x0, x1);
  const float e0 = expf(x0 - m), e1 = expf(x1 - m);
  const float s = e0 + e1;
  p0 = e0 / s;
  p1 = e1 / s;
}

// MARGIN: the input holds d = l1 - l0 per clip voxel ((n,32,H,W), logit_margin_kernel) instead of
// the two logit planes. softmax2(0, d) == softmax2(l0, l1) bit for bit: with m = max(l0, l1) one
// exponent is expf(0) and the other expf(-|d|), where fl(l0 - l1) == -fl(l1 - l0) exactly.
template <bool MARGIN>
__global__ void pass_labels_kernel(const float* __restrict__ logits, PassTable tab, int T, int step, int HW,
                                   int interp, uint8_t* __restrict__ labels) {
  const int k = blockIdx.z, f = blockIdx.y;
  const int tk = T - k * step;
  if (f >= tk) return;
  const int tc = 32 * round_half_even_div32(tk);
  const bool resample = interp && (tk & 31) && tk != tc;
  Lin L = {f, f, 1.f, 0.f};
  if (resample) L = lin_ac_false(tc, tk, f);
  const size_t clip_stride = (size_t)(MARGIN ? 1 : 2) * 32 * HW;
  const float* base = logits + (size_t)tab.clip0[k] * clip_stride;
  const float* a = base + (size_t)(L.i0 >> 5) * clip_stride + (size_t)(L.i0 & 31) * HW;
  const float* b = base + (size_t)(L.i1 >> 5) * clip_stride + (size_t)(L.i1 & 31) * HW;
  const size_t cs = (size_t)32 * HW;  // class stride inside a clip
  uint8_t* out = labels + ((size_t)k * T + f) * HW;
  if ((HW & 3) == 0 && ((uintptr_t)logits & 15) == 0 && ((uintptr_t)labels & 3) == 0) {
    // 4 pixels per thread: 16-B logit loads, one 4-byte label store
    auto lab = [&](float xa0, float xa1, float xb0, float xb1) __attribute__((always_inline)) {
      float pa0, pa1;
      softmax2(xa0, xa1, pa0, pa1);
      float q0 = pa0, q1 = pa1;
      if (resample) {
        float pb0, pb1;
        softmax2(xb0, xb1, pb0, pb1);
        q0 = lerp_t(pa0, pb0, L.l0, L.l1);
        q1 = lerp_t(pa1, pb1, L.l0, L.l1);
      }
      return (unsigned)(q1 > q0 ? 1 : 0);  // np.argmax: first maximum wins ties
    };
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (HW >> 2); i += gridDim.x * blockDim.x) {
      const f32x4 a0 = reinterpret_cast<const f32x4*>(a)[i];
      const f32x4 a1 = MARGIN ? a0 : reinterpret_cast<const f32x4*>(a + cs)[i];
      f32x4 b0 = a0, b1 = a1;
      if (resample) {
        b0 = reinterpret_cast<const f32x4*>(b)[i];
        b1 = MARGIN ? b0 : reinterpret_cast<const f32x4*>(b + cs)[i];
      }
      unsigned w = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w |= (MARGIN ? lab(0.f, a0[e], 0.f, b0[e]) : lab(a0[e], a1[e], b0[e], b1[e])) << (8 * e);
      reinterpret_cast<unsigned*>(out)[i] = w;
    }
    return;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x) {
    float pa0, pa1;
    if (MARGIN)
      softmax2(0.f, a[i], pa0, pa1);
    else
      softmax2(a[i], a[i + cs], pa0, pa1);
    float q0 = pa0, q1 = pa1;
    if (resample) {
      float pb0, pb1;
      if (MARGIN)
        softmax2(0.f, b[i], pb0, pb1);
      else
        softmax2(b[i], b[i + cs], pb0, pb1);
      q0 = lerp_t(pa0, pb0, L.l0, L.l1);
      q1 = lerp_t(pa1, pb1, L.l0, L.l1);
    }
    out[i] = q1 > q0 ? 1 : 0;  // np.argmax: first maximum wins ties
  }
}

// (n,2,32,HW) logits -> (n,32,HW) margins d = l1 - l0, 4 voxels per thread.
__global__ void logit_margin_kernel(const float* __restrict__ logits, int n, size_t per_clip,
                                    float* __restrict__ margin) {
  const size_t total4 = (size_t)n * per_clip / 4;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < total4; g += (size_t)gridDim.x * blockDim.x) {
    const size_t e = 4 * g, c = e / per_clip, r = e - c * per_clip;
    const float* l = logits + 2 * c * per_clip + r;
    const f32x4 l0 = *reinterpret_cast<const f32x4*>(l);
    const f32x4 l1 = *reinterpret_cast<const f32x4*>(l + per_clip);
    *reinterpret_cast<f32x4*>(margin + e) = l1 - l0;
  }
}

// ---- fuse_votes: majority ----------------------------------------------------------------------
// Output frame o: o == 0 -> frame 0 of pass 0; o >= 1 -> frame i = o + step - 1.
__device__ inline int n_votes(int i, int K, int step) {
  int nv = 0;
  const int kmax = min(i, K);
  for (int idx = 0; idx < kmax; ++idx) {
    if (i - idx * step < 0) break;
    ++nv;
  }
  return nv;
}

// Majority: ties -> background (0). ITK voting (itk::LabelVotingImageFilter with its default
// undecided label, max input label + 1): ties -> 2 (a tie of two labels needs both present, so the
// frame's max label is 1). PARITY UNPINNED: LabelFusion / SimpleITK are not available.
__global__ void fuse_majority_kernel(const uint8_t* __restrict__ labels, int K, int T, int step, int HW,
                                     uint8_t tie_label, uint8_t* __restrict__ fused) {
  const int o = blockIdx.y;
  const int i = o == 0 ? 0 : o + step - 1;
  const int nv = o == 0 ? 1 : n_votes(i, K, step);
  uint8_t* out = fused + (size_t)o * HW;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    int ones = 0;
    for (int idx = 0; idx < nv; ++idx) ones += labels[((size_t)idx * T + (i - idx * step)) * HW + p];
    out[p] = (nv == 1) ? (uint8_t)ones : 2 * ones == nv ? tie_label : (uint8_t)(2 * ones > nv ? 1 : 0);
  }
}

// ---- fuse_votes: SIMPLE (one workgroup per output frame) --------------------------------------
// Selective and iterative method for performance level estimation (Langerak et al. 2010) in the
// BraTS-toolkit form: per label (1 then 0), weighted majority of the binarised candidates with
// weights (dice(candidate, estimate) + 1)^2, drop candidates below 0.05 * max weight, stop when the
// estimate's voxel count moves by < 25. PARITY UNPINNED: LabelFusion's source is not available.
constexpr int SIMPLE_THREADS = 256;

__device__ inline double block_sum(double v, double* red) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0;
  for (int w = 0; w < SIMPLE_THREADS / 64; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(SIMPLE_THREADS) void fuse_simple_kernel(const uint8_t* __restrict__ labels, int K, int T,
                                                                      int step, int HW, uint8_t* __restrict__ fused) {
  extern __shared__ uint8_t est[];  // HW bytes: current estimate
  __shared__ double red[SIMPLE_THREADS / 64];
  __shared__ double wts[CLASFV_MAX_PASSES];
  const int o = blockIdx.x;
  const int i = o == 0 ? 0 : o + step - 1;
  const int nv = o == 0 ? 1 : n_votes(i, K, step);
  uint8_t* out = fused + (size_t)o * HW;
  auto vote = [&](int idx, int p) -> int { return labels[((size_t)idx * T + (i - idx * step)) * HW + p]; };
  if (nv == 1) {
    for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS) out[p] = (uint8_t)vote(0, p);
    return;
  }
  for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS) out[p] = 0;
  for (int lab = 1; lab >= 0; --lab) {
    uint64_t keep = (nv >= 64) ? ~0ull : ((1ull << nv) - 1ull);
    for (int idx = 0; idx < nv; ++idx) wts[idx] = 1.0;
    __syncthreads();
    // initial estimate: unweighted majority, ties -> off
    double cnt = 0;
    for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS) {
      double on = 0, off = 0;
      for (int idx = 0; idx < nv; ++idx) {
        const bool c = vote(idx, p) == lab;
        on += c ? 1.0 : 0.0;
        off += c ? 0.0 : 1.0;
      }
      est[p] = on > off;
      cnt += est[p];
    }
    double conv = block_sum(cnt, red);
    for (int it = 0; it < 25; ++it) {
      // dice of every kept candidate against the estimate
      double esum = conv;
      double mx = 0;
      for (int idx = 0; idx < nv; ++idx) {
        if (!(keep >> idx & 1ull)) continue;
        double inter = 0, csum = 0;
        for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS) {
          const bool c = vote(idx, p) == lab;
          csum += c;
          inter += (c && est[p]);
        }
        inter = block_sum(inter, red);
        csum = block_sum(csum, red);
        const double s = csum + esum;
        const double d = (s == 0) ? 1.0 : 2.0 * inter / s;
        const double w = (d + 1.0) * (d + 1.0);
        if (threadIdx.x == 0) wts[idx] = w;
        mx = fmax(mx, w);
      }
      __syncthreads();
      for (int idx = 0; idx < nv; ++idx)
        if ((keep >> idx & 1ull) && !(wts[idx] > 0.05 * mx)) keep &= ~(1ull << idx);
      cnt = 0;
      for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS) {
        double on = 0, off = 0;
        for (int idx = 0; idx < nv; ++idx) {
          if (!(keep >> idx & 1ull)) continue;
          const bool c = vote(idx, p) == lab;
          if (c)
            on += wts[idx];
          else
            off += wts[idx];
        }
        est[p] = on > off;
        cnt += est[p];
      }
      const double nsum = block_sum(cnt, red);
      const bool stop = fabs(conv - nsum) < 25.0;
      conv = nsum;
      if (stop) break;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < HW; p += SIMPLE_THREADS)
      if (est[p]) out[p] = (uint8_t)lab;
    __syncthreads();
  }
}

// Fast SIMPLE for <= 16 votes: the same iteration, with each pixel's votes packed once into a 16-bit
// mask in LDS, integer counts (exact: the Dice values and weights are those of the kernel above) and
// one block reduction per iteration (the candidate sizes are fixed per label; the overlaps with the
// new estimate are accumulated in the pass that computes it). 1024 threads per output frame. All
// per-candidate loops run to the compile-time bound (guarded by nv) so the arrays stay in registers.
constexpr int SIMPLE_FAST_THREADS = 1024;
constexpr int SIMPLE_FAST_MAXV = 16;

// Block sum of N ints per thread; every thread gets the totals in tot[].
template <int N>
__device__ inline void block_sum_vec(const int (&v)[N], int (*red)[2 * SIMPLE_FAST_MAXV + 1], int* tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    int x = v[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if (lane == 0) red[wid][j] = x;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < SIMPLE_FAST_THREADS / 64; ++w) t += red[w][threadIdx.x];
    tot[threadIdx.x] = t;
  }
  __syncthreads();
}

__global__ __launch_bounds__(SIMPLE_FAST_THREADS) void fuse_simple_fast_kernel(const uint8_t* __restrict__ labels, int K,
                                                                               int T, int step, int HW,
                                                                               uint8_t* __restrict__ fused) {
  constexpr int MV = SIMPLE_FAST_MAXV;
  extern __shared__ uint8_t smem_simple[];
  uint16_t* msk = reinterpret_cast<uint16_t*>(smem_simple);  // bit idx: vote idx == 1
  uint8_t* est = smem_simple + 2 * (size_t)HW;                // bit 0: current estimate, bit 1: label-1 result
  __shared__ int red[SIMPLE_FAST_THREADS / 64][2 * MV + 1];
  __shared__ int tot[2 * MV + 1];
  const int o = blockIdx.x;
  const int i = o == 0 ? 0 : o + step - 1;
  const int nv = o == 0 ? 1 : n_votes(i, K, step);
  uint8_t* out = fused + (size_t)o * HW;
  if (nv == 1) {
    for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) out[p] = labels[(size_t)i * HW + p];
    return;
  }
  const unsigned full = (1u << nv) - 1u;
  for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) {
    unsigned m = 0;
    for (int idx = 0; idx < nv; ++idx) m |= (unsigned)(labels[((size_t)idx * T + (i - idx * step)) * HW + p] != 0) << idx;
    msk[p] = (uint16_t)m;
    est[p] = 0;
  }
  __syncthreads();
  for (int lab = 1; lab >= 0; --lab) {
    unsigned keep = full;
    double wts[MV];
    int inter[MV], csum[MV];
    int conv;
    {
      // pass 0: unweighted majority (ties -> off), its size, its overlap with every candidate, and the
      // candidate sizes
      int acc[2 * MV + 1];
#pragma unroll
      for (int j = 0; j < 2 * MV + 1; ++j) acc[j] = 0;
      for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) {
        const unsigned c = lab ? msk[p] : (~(unsigned)msk[p] & full);
        const int on = __popc(c);
        const unsigned e = on > nv - on;
        est[p] = (uint8_t)((est[p] & 2u) | e);
        acc[0] += e;
#pragma unroll
        for (int idx = 0; idx < MV; ++idx) {
          const unsigned b = (c >> idx) & 1u;
          acc[1 + idx] += b & e;
          acc[1 + MV + idx] += b;
        }
      }
      block_sum_vec<2 * MV + 1>(acc, red, tot);
      conv = tot[0];
#pragma unroll
      for (int idx = 0; idx < MV; ++idx) {
        inter[idx] = tot[1 + idx];
        csum[idx] = tot[1 + MV + idx];
        wts[idx] = 1.0;
      }
      __syncthreads();
    }
    for (int it = 0; it < 25; ++it) {
      const double esum = (double)conv;
      double mx = 0;
#pragma unroll
      for (int idx = 0; idx < MV; ++idx) {
        if (idx >= nv || !(keep >> idx & 1u)) continue;
        const double s2 = (double)csum[idx] + esum;
        const double d = (s2 == 0) ? 1.0 : 2.0 * (double)inter[idx] / s2;
        wts[idx] = (d + 1.0) * (d + 1.0);
        mx = fmax(mx, wts[idx]);
      }
#pragma unroll
      for (int idx = 0; idx < MV; ++idx)
        if (idx < nv && (keep >> idx & 1u) && !(wts[idx] > 0.05 * mx)) keep &= ~(1u << idx);
      int acc[MV + 1];
#pragma unroll
      for (int j = 0; j < MV + 1; ++j) acc[j] = 0;
      for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) {
        const unsigned c = lab ? msk[p] : (~(unsigned)msk[p] & full);
        double on = 0, off = 0;
#pragma unroll
        for (int idx = 0; idx < MV; ++idx) {
          if (!(keep >> idx & 1u)) continue;  // keep has no bits at or above nv
          if ((c >> idx) & 1u)
            on += wts[idx];
          else
            off += wts[idx];
        }
        const unsigned e = on > off;
        est[p] = (uint8_t)((est[p] & 2u) | e);
        acc[0] += e;
#pragma unroll
        for (int idx = 0; idx < MV; ++idx) acc[1 + idx] += ((c >> idx) & 1u) & e;
      }
      block_sum_vec<MV + 1>(acc, red, tot);
      const int nsum = tot[0];
#pragma unroll
      for (int idx = 0; idx < MV; ++idx) inter[idx] = tot[1 + idx];
      __syncthreads();
      const bool stop = fabs((double)conv - (double)nsum) < 25.0;
      conv = nsum;
      if (stop) break;
    }
    if (lab == 1)
      for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) est[p] = (uint8_t)((est[p] & 1u) << 1);
    __syncthreads();
  }
  // label 1 where its estimate is on, then label 0 where its estimate is on (as the kernel above)
  for (int p = threadIdx.x; p < HW; p += SIMPLE_FAST_THREADS) out[p] = (uint8_t)((est[p] & 2u) && !(est[p] & 1u));
}

// ---- fuse_votes: STAPLE (one workgroup per output frame) --------------------------------------
// Simultaneous truth and performance level estimation (Warfield, Zou & Wells 2004), binary form as in
// ITK's STAPLEImageFilter: rater j's decision D_j = (vote == 1); prior f = mean of all D over raters
// and pixels; sensitivity p_j and specificity q_j start at 0.99999; E step W = f P1 / (f P1 + (1-f)
// P0) with P1 = prod_j (D_j ? p_j : 1 - p_j), P0 = prod_j (D_j ? 1 - q_j : q_j) (j ascending, double);
// M step p_j = sum W D_j / sum W, q_j = sum (1-W)(1-D_j) / sum (1-W) (a zero denominator keeps the
// old value); stop when no p_j, q_j moves by more than 1e-7 or after 100 iterations; label 1 where
// the final E step gives W > 0.5. PARITY UNPINNED (LabelFusion's source is not available); the
// oracle restates the same iteration in numpy (oracle/fuse_ref.py:staple_vote).
constexpr int STAPLE_THREADS = 1024;
constexpr int STAPLE_CHUNK = 16;  // raters accumulated per pass over the frame
constexpr int STAPLE_MAX_IT = 100;

__device__ inline double staple_w(unsigned long long d, int nv, const double* p, const double* q, double f) {
  double a = f, b = 1.0 - f;
  for (int j = 0; j < nv; ++j) {
    const bool on = (d >> j) & 1ull;
    a *= on ? p[j] : 1.0 - p[j];
    b *= on ? 1.0 - q[j] : q[j];
  }
  const double s = a + b;
  return s > 0.0 ? a / s : f;
}

// Block sum of N doubles per thread; totals land in tot[0..N).
template <int N>
__device__ inline void block_sum_dvec(const double (&v)[N], double (*red)[N], double* tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double x = v[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if (lane == 0) red[wid][j] = x;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    double t = 0.0;
    for (int w = 0; w < STAPLE_THREADS / 64; ++w) t += red[w][threadIdx.x];
    tot[threadIdx.x] = t;
  }
  __syncthreads();
}

__global__ __launch_bounds__(STAPLE_THREADS) void fuse_staple_kernel(const uint8_t* __restrict__ labels, int K, int T,
                                                                      int step, int HW, uint8_t* __restrict__ fused) {
  constexpr int NS = 2 * STAPLE_CHUNK + 1;
  __shared__ double red[STAPLE_THREADS / 64][NS];
  __shared__ double tot[NS];
  __shared__ double sp[CLASFV_MAX_PASSES], sq[CLASFV_MAX_PASSES], np_[CLASFV_MAX_PASSES], nq_[CLASFV_MAX_PASSES];
  __shared__ int s_done;
  const int o = blockIdx.x;
  const int i = o == 0 ? 0 : o + step - 1;
  const int nv = o == 0 ? 1 : n_votes(i, K, step);
  uint8_t* out = fused + (size_t)o * HW;
  auto votes = [&](int p) -> unsigned long long {
    unsigned long long d = 0;
    for (int j = 0; j < nv; ++j) d |= (unsigned long long)(labels[((size_t)j * T + (i - j * step)) * HW + p] == 1) << j;
    return d;
  };
  if (nv == 1) {
    for (int p = threadIdx.x; p < HW; p += STAPLE_THREADS) out[p] = labels[(size_t)i * HW + p];
    return;
  }
  // prior: fraction of foreground decisions over all raters and pixels
  {
    double c[NS];
    for (int j = 0; j < NS; ++j) c[j] = 0.0;
    for (int p = threadIdx.x; p < HW; p += STAPLE_THREADS) c[0] += (double)__popcll(votes(p));
    block_sum_dvec<NS>(c, red, tot);
  }
  const double f = tot[0] / ((double)nv * (double)HW);
  if (threadIdx.x < nv) sp[threadIdx.x] = sq[threadIdx.x] = 0.99999;
  __syncthreads();
  for (int it = 0; it < STAPLE_MAX_IT; ++it) {
    if (threadIdx.x == 0) s_done = 1;
    for (int j0 = 0; j0 < nv; j0 += STAPLE_CHUNK) {
      // acc[0] = sum W, acc[1 + j] = sum W D_j, acc[1 + C + j] = sum (1 - W)(1 - D_j)
      double acc[NS];
      for (int j = 0; j < NS; ++j) acc[j] = 0.0;
      for (int p = threadIdx.x; p < HW; p += STAPLE_THREADS) {
        const unsigned long long d = votes(p);
        const double w = staple_w(d, nv, sp, sq, f);
        acc[0] += w;
#pragma unroll
        for (int j = 0; j < STAPLE_CHUNK; ++j) {
          const bool on = (d >> (j0 + j)) & 1ull;  // bits at or past nv are 0
          acc[1 + j] += on ? w : 0.0;
          acc[1 + STAPLE_CHUNK + j] += on ? 0.0 : 1.0 - w;
        }
      }
      block_sum_dvec<NS>(acc, red, tot);
      const double sw = tot[0];
      const double sn = (double)HW - sw;  // sum (1 - W)
      if (threadIdx.x < STAPLE_CHUNK && j0 + threadIdx.x < nv) {
        const int j = j0 + threadIdx.x;
        np_[j] = sw > 0.0 ? tot[1 + threadIdx.x] / sw : sp[j];
        nq_[j] = sn > 0.0 ? tot[1 + STAPLE_CHUNK + threadIdx.x] / sn : sq[j];
        if (fabs(np_[j] - sp[j]) > 1e-7 || fabs(nq_[j] - sq[j]) > 1e-7) s_done = 0;
      }
      __syncthreads();  // tot is rewritten by the next chunk's reduction
    }
    // every E step of this iteration used the old p, q: publish the new ones
    if (threadIdx.x < nv) {
      sp[threadIdx.x] = np_[threadIdx.x];
      sq[threadIdx.x] = nq_[threadIdx.x];
    }
    __syncthreads();
    if (s_done) break;
    __syncthreads();  // s_done is reset at the top of the next iteration
  }
  for (int p = threadIdx.x; p < HW; p += STAPLE_THREADS) out[p] = staple_w(votes(p), nv, sp, sq, f) > 0.5 ? 1 : 0;
}

// ---- warp ------------------------------------------------------------------------------------
// torch.linspace(-1, 1, n) on the CPU: step = 2/(n-1); first half fma(step, i, -1), second half
// fma(-step, n-1-i, 1) (the kernel is built with FMA contraction).
__device__ inline float linspace_pm1(int i, int n) {
  if (n == 1) return -1.f;
  const float step = 2.0f / (float)(n - 1);
  return (i < n / 2) ? fmaf(step, (float)i, -1.f) : fmaf(-step, (float)(n - 1 - i), 1.f);
}

// F.grid_sample(bilinear, border, align_corners=False) as PyTorch's vectorised CPU kernel computes it
// (GridSamplerKernel.cpp, built with FMA contraction; bit-exact vs the reference golden):
// ix = fma(gx + 1, W/2, -0.5) clipped to [0, W-1]; corner weights nw = s*e, ne = s*w, sw = n*e, se = n*w
// with w = ix - floor(ix), e = floor(ix) + 1 - ix (same in y); value = fma(se_v, se, fma(sw_v, sw,
// fma(ne_v, ne, nw_v * nw))), out-of-range corners read as 0.
__global__ void warp_kernel(const float* __restrict__ img, int N, int C, int H, int W, const float* __restrict__ motion,
                            int64_t m_sn, int64_t m_sc, float* __restrict__ out) {
  const size_t HW = (size_t)H * W;
  const size_t total = (size_t)N * HW;
  const float sx = (float)W * 0.5f, sy = (float)H * 0.5f;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < total; g += (size_t)gridDim.x * blockDim.x) {
    const int n = (int)(g / HW);
    const int pix = (int)(g - (size_t)n * HW);
    const int i = pix / W, j = pix - (pix / W) * W;
    const float* mp = motion + n * m_sn + pix;
    const float gx = linspace_pm1(j, W) + mp[0];
    const float gy = linspace_pm1(i, H) + mp[m_sc];
    const float ix = fminf((float)(W - 1), fmaxf(fmaf(gx + 1.f, sx, -0.5f), 0.f));
    const float iy = fminf((float)(H - 1), fmaxf(fmaf(gy + 1.f, sy, -0.5f), 0.f));
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    const float we = ix - fx0, ee = (fx0 + 1.f) - ix, wn = iy - fy0, ws = (fy0 + 1.f) - iy;
    const float wnw = ws * ee, wne = ws * we, wsw = wn * ee, wse = wn * we;
    const bool in_x1 = x1 < W, in_y1 = y1 < H;
    for (int c = 0; c < C; ++c) {
      const float* src = img + ((size_t)n * C + c) * HW;
      const float vnw = src[y0 * W + x0];
      const float vne = in_x1 ? src[y0 * W + x1] : 0.f;
      const float vsw = in_y1 ? src[y1 * W + x0] : 0.f;
      const float vse = (in_x1 && in_y1) ? src[y1 * W + x1] : 0.f;
      out[((size_t)n * C + c) * HW + pix] = fmaf(vse, wse, fmaf(vsw, wsw, fmaf(vne, wne, vnw * wnw)));
    }
  }
}

// Backward of warp_kernel (grid_sampler_2d_backward, bilinear, border, align_corners=False, as
// PyTorch's vectorised CPU kernel): per output pixel and channel, grad_img gets gOut * corner
// weight at the four corners (float atomics: the summation order differs from the CPU's sequential
// scatter, so grad_img matches to rounding, not bit for bit); the motion gradient accumulates
// fma(se_v - sw_v, n, (ne_v - nw_v) * s) * gOut (x) and fma(se_v - ne_v, w, (sw_v - nw_v) * e) * gOut
// (y) over channels, times W/2 (H/2) when the unclipped source coordinate lies strictly inside
// (0, W-1), else 0 (border clipping kills the gradient) -- bit-exact vs the CPU kernel.
__global__ void warp_backward_kernel(const float* __restrict__ gout, const float* __restrict__ img, int N, int C, int H,
                                     int W, const float* __restrict__ motion, int64_t m_sn, int64_t m_sc,
                                     float* __restrict__ gimg, float* __restrict__ gmot) {
  const size_t HW = (size_t)H * W;
  const size_t total = (size_t)N * HW;
  const float sx = (float)W * 0.5f, sy = (float)H * 0.5f;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < total; g += (size_t)gridDim.x * blockDim.x) {
    const int n = (int)(g / HW);
    const int pix = (int)(g - (size_t)n * HW);
    const int i = pix / W, j = pix - (pix / W) * W;
    const float* mp = motion + n * m_sn + pix;
    const float gx = linspace_pm1(j, W) + mp[0];
    const float gy = linspace_pm1(i, H) + mp[m_sc];
    const float ux = fmaxf(fmaf(gx + 1.f, sx, -0.5f), 0.f), uy = fmaxf(fmaf(gy + 1.f, sy, -0.5f), 0.f);
    const float ix = fminf(ux, (float)(W - 1)), iy = fminf(uy, (float)(H - 1));
    const float mx = (ux != 0.f && ix != (float)(W - 1)) ? sx : 0.f;
    const float my = (uy != 0.f && iy != (float)(H - 1)) ? sy : 0.f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    const float we = ix - fx0, ee = (fx0 + 1.f) - ix, wn = iy - fy0, ws = (fy0 + 1.f) - iy;
    const float wnw = ws * ee, wne = ws * we, wsw = wn * ee, wse = wn * we;
    const bool in_x1 = x1 < W, in_y1 = y1 < H;
    float ax = 0.f, ay = 0.f;
    for (int c = 0; c < C; ++c) {
      const size_t plane = ((size_t)n * C + c) * HW;
      const float go = gout[plane + pix];
      const float* src = img + plane;
      const float vnw = src[y0 * W + x0];
      const float vne = in_x1 ? src[y0 * W + x1] : 0.f;
      const float vsw = in_y1 ? src[y1 * W + x0] : 0.f;
      const float vse = (in_x1 && in_y1) ? src[y1 * W + x1] : 0.f;
      if (gimg) {
        float* d = gimg + plane;
        atomicAdd(d + y0 * W + x0, go * wnw);
        if (in_x1) atomicAdd(d + y0 * W + x1, go * wne);
        if (in_y1) atomicAdd(d + y1 * W + x0, go * wsw);
        if (in_x1 && in_y1) atomicAdd(d + y1 * W + x1, go * wse);
      }
      ax = fmaf(fmaf(vse - vsw, wn, (vne - vnw) * ws), go, ax);
      ay = fmaf(fmaf(vse - vne, we, (vsw - vnw) * ee), go, ay);
    }
    if (gmot) {
      gmot[(size_t)n * 2 * HW + pix] = ax * mx;
      gmot[((size_t)n * 2 + 1) * HW + pix] = ay * my;
    }
  }
}

// ---- preprocess_video ---------------------------------------------------------------------------
// motion_segment.py:96-106: (T,Hs,Ws,3) uint8 RGB frames -> (3,T,Hs,Ws) float32 -> F.interpolate(
// size=(T,H,W), mode="trilinear", align_corners=True). T is unchanged, so the temporal weights are
// (1, 0) and that level is the identity; per spatial axis PyTorch's CPU kernel computes
// src = scale * dst with scale = (float)(in-1)/(out-1), i0 = min((int)src, in-1), l1 = clamp(src - i0),
// l0 = 1 - l1, and combines W first, then H, as fma(x0, l0, x1 * l1) at each level (bit-exact vs
// F.interpolate on the CPU; tests/test_oracle.py, tests/test_gpu.py).
__device__ inline Lin lin_ac_true(int n_in, float scale, int dst) {
  Lin r;
  const float src = (scale * (float)dst);
  r.i0 = min((int)src, n_in - 1);
  r.l1 = fminf(fmaxf((src - (float)r.i0), 0.f), 1.f);
  r.i1 = r.i0 + (r.i0 < n_in - 1 ? 1 : 0);
  r.l0 = (1.f - r.l1);
  return r;
}

__global__ void preprocess_video_kernel(const uint8_t* __restrict__ frames, int T, int Hs, int Ws, int H, int W,
                                        float sh, float sw, float* __restrict__ out) {
  const int t = blockIdx.z, y = blockIdx.y;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= W) return;
  const Lin ly = lin_ac_true(Hs, sh, y), lx = lin_ac_true(Ws, sw, x);
  const uint8_t* f = frames + (size_t)t * Hs * Ws * 3;
  const uint8_t* r0 = f + (size_t)ly.i0 * Ws * 3;
  const uint8_t* r1 = f + (size_t)ly.i1 * Ws * 3;
  const size_t plane = (size_t)T * H * W;
  float* o = out + ((size_t)t * H + y) * W + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float a = r0[lx.i0 * 3 + c], b = r0[lx.i1 * 3 + c];
    const float cc = r1[lx.i0 * 3 + c], d = r1[lx.i1 * 3 + c];
    const float top = lerp_t(a, b, lx.l0, lx.l1);
    const float bot = lerp_t(cc, d, lx.l0, lx.l1);
    o[c * plane] = lerp_t(top, bot, ly.l0, ly.l1);
  }
}

// ---- zeroone_normalize -------------------------------------------------------------------------
constexpr int RED_THREADS = 256, RED_BLOCKS = 512;

__global__ void minmax_partial_kernel(const float* __restrict__ v, int64_t n, float* __restrict__ part) {
  const int c = blockIdx.y;
  const float* x = v + (size_t)c * n;
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int64_t i = blockIdx.x * (int64_t)RED_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * RED_THREADS) {
    lo = fminf(lo, x[i]);
    hi = fmaxf(hi, x[i]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, off, 64));
    hi = fmaxf(hi, __shfl_xor(hi, off, 64));
  }
  __shared__ float slo[RED_THREADS / 64], shi[RED_THREADS / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    slo[wid] = lo;
    shi[wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < RED_THREADS / 64; ++w) {
      lo = fminf(lo, slo[w]);
      hi = fmaxf(hi, shi[w]);
    }
    part[(c * gridDim.x + blockIdx.x) * 2] = lo;
    part[(c * gridDim.x + blockIdx.x) * 2 + 1] = hi;
  }
}

__global__ void normalize_kernel(float* __restrict__ v, int64_t n, const float* __restrict__ part, int nparts) {
  const int c = blockIdx.y;
  __shared__ float s_lo, s_den;
  if (threadIdx.x == 0) {
    float lo = FLT_MAX, hi = -FLT_MAX;
    for (int b = 0; b < nparts; ++b) {
      lo = fminf(lo, part[(c * nparts + b) * 2]);
      hi = fmaxf(hi, part[(c * nparts + b) * 2 + 1]);
    }
    s_lo = lo;
    s_den = (hi - lo);  // == max over the channel of (x - min): subtraction is monotone
  }
  __syncthreads();
  const float lo = s_lo, den = s_den;
  float* x = v + (size_t)c * n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = ((x[i] - lo) / den);
}

inline int blocks_for(size_t n, int per_block, int cap) {
  size_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return (int)(b > (size_t)cap ? cap : b);
}

}  // namespace

hipError_t launch_build_clips(const float* video, int T, int HW, const int32_t* table, int n, int interp, float* clips,
                              hipStream_t s) {
  dim3 grid(blocks_for(HW % 4 ? HW : HW / 4, 256, 64), 3 * 32, n);
  hipLaunchKernelGGL(build_clips_kernel, grid, dim3(256), 0, s, video, T, HW, table, interp, clips);
  return hipGetLastError();
}

hipError_t launch_pass_labels(const float* logits, int K, const int32_t* clip0, int T, int step, int HW, int interp,
                              int margin, uint8_t* labels, hipStream_t s) {
  PassTable tab;
  for (int k = 0; k < K; ++k) tab.clip0[k] = clip0[k];
  dim3 grid(blocks_for(HW % 4 ? HW : HW / 4, 256, 64), T, K);
  if (margin)
    hipLaunchKernelGGL(pass_labels_kernel<true>, grid, dim3(256), 0, s, logits, tab, T, step, HW, interp, labels);
  else
    hipLaunchKernelGGL(pass_labels_kernel<false>, grid, dim3(256), 0, s, logits, tab, T, step, HW, interp, labels);
  return hipGetLastError();
}

hipError_t launch_logit_margin(const float* logits, int n, int HW, float* margin, hipStream_t s) {
  const size_t per_clip = (size_t)32 * HW;  // a multiple of 4: 16-B vectors never straddle clips
  hipLaunchKernelGGL(logit_margin_kernel, dim3(blocks_for((size_t)n * per_clip / 4, 256, 8192)), dim3(256), 0, s, logits,
                     n, per_clip, margin);
  return hipGetLastError();
}

hipError_t launch_fuse_votes(const uint8_t* labels, int K, int T, int step, int HW, int method, uint8_t* fused,
                             hipStream_t s) {
  const int tout = T - (step - 1);
  const bool force_generic = (method & CLASFV_FUSE_FORCE_GENERIC) != 0;  // A/B testing of the SIMPLE kernels
  method &= ~CLASFV_FUSE_FORCE_GENERIC;
  if (method == 2) {
    hipLaunchKernelGGL(fuse_staple_kernel, dim3(tout), dim3(STAPLE_THREADS), 0, s, labels, K, T, step, HW, fused);
  } else if (method == 1) {
    const size_t lds = 3 * (size_t)HW;
    if (K <= SIMPLE_FAST_MAXV && lds <= 160 * 1024 && !force_generic) {
      static size_t attr = 0;
      if (lds > 64 * 1024 && lds > attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fuse_simple_fast_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = lds;
      }
      hipLaunchKernelGGL(fuse_simple_fast_kernel, dim3(tout), dim3(SIMPLE_FAST_THREADS), lds, s, labels, K, T, step, HW,
                         fused);
    } else {
      hipLaunchKernelGGL(fuse_simple_kernel, dim3(tout), dim3(SIMPLE_THREADS), HW, s, labels, K, T, step, HW, fused);
    }
  } else {
    dim3 grid(blocks_for(HW, 256, 64), tout);
    const uint8_t tie = method == 3 ? 2 : 0;  // CLASFV_FUSE_ITKVOTING
    hipLaunchKernelGGL(fuse_majority_kernel, grid, dim3(256), 0, s, labels, K, T, step, HW, tie, fused);
  }
  return hipGetLastError();
}

hipError_t launch_warp(const float* img, int N, int C, int H, int W, const float* motion, int64_t m_sn, int64_t m_sc,
                       float* out, hipStream_t s) {
  const size_t total = (size_t)N * H * W;
  hipLaunchKernelGGL(warp_kernel, dim3(blocks_for(total, 256, 8192)), dim3(256), 0, s, img, N, C, H, W, motion, m_sn,
                     m_sc, out);
  return hipGetLastError();
}

hipError_t launch_warp_backward(const float* gout, const float* img, int N, int C, int H, int W, const float* motion,
                                int64_t m_sn, int64_t m_sc, float* gimg, float* gmot, hipStream_t s) {
  const size_t total = (size_t)N * H * W;
  hipLaunchKernelGGL(warp_backward_kernel, dim3(blocks_for(total, 256, 8192)), dim3(256), 0, s, gout, img, N, C, H, W,
                     motion, m_sn, m_sc, gimg, gmot);
  return hipGetLastError();
}

hipError_t launch_zeroone_normalize(float* v, int64_t n, float* part, hipStream_t s) {
  const int nb = blocks_for((size_t)n, RED_THREADS * 4, RED_BLOCKS);
  hipLaunchKernelGGL(minmax_partial_kernel, dim3(nb, 3), dim3(RED_THREADS), 0, s, v, n, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(normalize_kernel, dim3(blocks_for((size_t)n, 1024, 2048), 3), dim3(256), 0, s, v, n, part, nb);
  return hipGetLastError();
}

int zeroone_partials_floats() { return 3 * RED_BLOCKS * 2; }

hipError_t launch_preprocess_video(const uint8_t* frames, int T, int Hs, int Ws, int H, int W, float* out,
                                   hipStream_t s) {
  // align_corners=True scales in host float arithmetic, as at::native::area_pixel_compute_scale
  const float sh = H > 1 ? (float)(Hs - 1) / (float)(H - 1) : 0.f;
  const float sw = W > 1 ? (float)(Ws - 1) / (float)(W - 1) : 0.f;
  dim3 grid((W + 127) / 128, H, T);
  hipLaunchKernelGGL(preprocess_video_kernel, grid, dim3(128), 0, s, frames, T, Hs, Ws, H, W, sh, sw, out);
  return hipGetLastError();
}
