// conv_twalk_bf16 (round 6): the bf16 engines' stride-1 temporal 3x1x1 convs with 64 output channels
// -- the Conv2Plus1D second halves of layer1 (torchvision Conv2Plus1D via
// src/model/R2plus1D_18_MotionNet.py:31, 144 -> 64 channels, padded 160 -> 64) and the stem's
// temporal conv (45 -> 64, padded 64 -> 64; :29) -- as a frame-walking stream.
//
// conv_patch_bf16 runs these as 4-frame x 64-pixel blocks: each block stages a 6-frame patch (a 1.5x
// temporal halo), runs 15 K steps and stores; every block's load / compute / store phases are in
// lockstep with every other block's, so HBM idles while the chip computes and the MFMAs idle while it
// stores. Here one wave owns a 32-pixel column of one clip and walks a 16- (or 8-) frame segment of it:
//  * input-stationary: input frame u is read ONCE (halo only at segment ends: 18 frames per 16 outputs)
//    and feeds its three outputs, y[u+1] += W0 x[u], y[u] += W1 x[u], y[u-1] += W2 x[u]; three rolling
//    32x64 fp32 accumulators (96 VGPRs), after frame u output u-1 is complete and stored;
//  * no LDS ring and no block barrier in the loop: a frame's B operands (32 pixels x Cin bf16, lane =
//    pixel, 8 channels per 16-B load) are loaded straight into registers two frames ahead (a 3-frame
//    register ring), so every wave always has its next two frames' loads and its last output's stores
//    in flight -- loads, MFMAs and stores of different frames overlap inside each wave;
//  * the weights (64 x 3 Cin bf16, conv_dma's image w[n][tap Cin + c]) are copied to LDS once per
//    block with an odd 16-B row pitch (the 32-row A fragments of v_mfma_f32_32x32x16_bf16 hit 16
//    distinct bank quads per ds_read_b128 lane group) and read as the A operand: 6 fragments per 16
//    input channels feed 6 MFMAs;
//  * D = W . X^T: lane (pixel r, half h) holds channels 32 rb + 8 g + 4 h .. + 3 of pixel r, so the
//    epilogue (folded-BN bias, residual, ReLU) stores 8-B bf16 vectors.
// K order per output: input frame, then 16-channel step, then tap -- not conv_patch_bf16's, so outputs
// match it within bf16 rounding, not bit for bit.
#include <hip/hip_bf16.h>

#include <utility>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int TW_PX = 32;  // pixels per wave (one 32-column MFMA block)

__host__ __device__ constexpr int tw_pitch(int cin) {  // LDS row pitch (bytes) of the weights: odd 16-B count
  return (6 * cin / 16) % 2 == 0 ? 6 * cin + 16 : 6 * cin;
}

template <int... I, class F>
__device__ inline void tw_unroll(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

// CS = Cin / 16 (16-channel K steps per tap), TS = output frames per wave segment, EF bit 0 residual,
// bit 1 ReLU, PD = input frames loaded ahead (register ring of PD + 1 frames), W = waves per SIMD
// KO (convbench knock-outs, wrong results): 1 no output stores, 2 no input loads in the walk, 4 no MFMAs
constexpr int TW_SP = 144;  // staging row pitch (bytes): 128 + 16, conflict-free 8-B accesses of 32 rows
template <int CS, int TS, int EF, int PD, int W, int KO = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) void conv_twalk_bf16(ConvParams p, int n_cols,
                                                                                                   int n_seg) {
  constexpr int CIN = 16 * CS, KP = 3 * CIN, PITCH = tw_pitch(CIN);
  constexpr int NI = TS + 2;  // input frames per segment (one halo frame each side)
  extern __shared__ __align__(16) char smem[];  // [64 rows][PITCH] weights, 64 fp32 biases, staging
  float* sbias = reinterpret_cast<float*>(smem + 64 * PITCH);
  char* stg = smem + 64 * PITCH + 256 + (threadIdx.x >> 6) * 32 * TW_SP;  // this wave's staging rows

  const int tid = threadIdx.x, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  // weights -> LDS once per block (16-B chunks, row pitch PITCH)
  {
    const char* w = reinterpret_cast<const char*>(p.w);
    constexpr int CPR = KP * 2 / 16;  // 16-B chunks per weight row
    for (int c = tid; c < 64 * CPR; c += 256) {
      const int row = c / CPR, k = c - row * CPR;
      *reinterpret_cast<f32x4*>(smem + row * PITCH + k * 16) =
          *reinterpret_cast<const f32x4*>(w + ((size_t)row * KP) * 2 + k * 16);
    }
    if (tid < 64) sbias[tid] = p.bias[tid];
  }
  __syncthreads();

  // this wave's (clip, 32-pixel column, frame segment)
  const int HW = p.Hi * p.Wi, T = p.Ti;
  int item = blockIdx.x * 4 + (tid >> 6);
  const int seg = item % n_seg;
  item /= n_seg;
  const int col = item % n_cols, clip = item / n_cols;
  if (clip >= p.N) return;  // (the grid is whole blocks of 4 waves; no barrier follows)
  const int ta = seg * TS;
  const int px = col * TW_PX + r;
  const bool pv = px < HW;  // lanes past the map load pixel 0 (their outputs are not stored)
  const __bf16* x = reinterpret_cast<const __bf16*>(p.x) + ((size_t)clip * T * HW + (pv ? px : 0)) * CIN + 8 * h;
  const size_t frame_x = (size_t)HW * CIN;
  // the column's pixel 0 in the output and the residual
  __bf16* ybase = reinterpret_cast<__bf16*>(p.y) + ((size_t)clip * T * HW + col * TW_PX) * 64;
  const __bf16* rbase = reinterpret_cast<const __bf16*>(p.res) + ((size_t)clip * T * HW + col * TW_PX) * 64;
  const size_t frame_y = (size_t)HW * 64;

  constexpr int NR = PD + 1;
  bf16x8 xr[NR][CS];  // register ring: input frame ta - 1 + i in slot i % NR
  f32x16 acc[3][2];  // rolling outputs: y[u - 1], y[u], y[u + 1] of input frame u in slots (i+2)%3, i%3... (below)
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  auto load_frame = [&](int u, bf16x8 (&dst)[CS]) __attribute__((always_inline)) {
    if ((KO & 2) && u > ta + 1) return;
    if (u >= 0 && u < T) {  // wave-uniform; frames outside the clip are zero padding (never read)
      const __bf16* src = x + (size_t)u * frame_x;
#pragma unroll
      for (int s = 0; s < CS; ++s) dst[s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
    }
  };
  // A fragment (weights) of tap kt, 16-channel step s, row block rb: row 32 rb + r, k 16 s + 8 h
  const char* wa = smem + r * PITCH + (8 * h) * 2;
  auto wfrag = [&](int kt, int s, int rb) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8*>(wa + (32 * rb) * PITCH + (kt * CIN + 16 * s) * 2);
  };

#pragma unroll
  for (int i = 0; i < PD; ++i) load_frame(ta - 1 + i, xr[i]);

  // Output (and residual) rows go through the wave's LDS staging rows: a store / load instruction then
  // moves 8 whole 128-B pixel rows (lane: row 8 k + lane / 8, 16-B slot lane % 8) instead of 8-B pieces
  // of 32 rows. The residual of output frame o is loaded one step before its epilogue (double-buffered,
  // 4 x 16 B per lane).
  f32x4 rvq[2][4];
  auto load_res = [&](int o, f32x4 (&rq)[4]) __attribute__((always_inline)) {
    if constexpr (EF & 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = 8 * k + (lane >> 3), sl = lane & 7;
        rq[k] = col * TW_PX + row < HW ? *reinterpret_cast<const f32x4*>(rbase + (size_t)o * frame_y + (size_t)row * 64 + sl * 8)
                                       : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto wave_sync = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  };
  // output frame o of accumulator slot ac: bias, residual, ReLU, bf16; the slot is cleared
  auto store_out = [&](int o, f32x16 (&ac)[2], const f32x4 (&rq)[4]) __attribute__((always_inline)) {
    if constexpr (EF & 1) {  // the residual rows into the staging rows (each element's own address below)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        *reinterpret_cast<f32x4*>(stg + (8 * k + (lane >> 3)) * TW_SP + (lane & 7) * 16) = rq[k];
      wave_sync();
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        char* e = stg + r * TW_SP + (32 * rb + 8 * g + 4 * h) * 2;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + 32 * rb + 8 * g + 4 * h);
        f32x4 v = {ac[rb][4 * g] + bv[0], ac[rb][4 * g + 1] + bv[1], ac[rb][4 * g + 2] + bv[2], ac[rb][4 * g + 3] + bv[3]};
        if constexpr (EF & 1) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(e);
          v += f32x4{(float)rv[0], (float)rv[1], (float)rv[2], (float)rv[3]};
        }
        if constexpr (EF & 2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = relu1(v[q]);
        }
        const bf16x4 ov = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        if constexpr (KO & 1) {
          if ((float)ov[0] == 12345.f) *reinterpret_cast<bf16x4*>(e) = ov;  // (knock-out: no stores)
        } else {
          *reinterpret_cast<bf16x4*>(e) = ov;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) ac[rb][4 * g + q] = 0.f;
      }
    if constexpr (!(KO & 1)) {
      wave_sync();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = 8 * k + (lane >> 3), sl = lane & 7;
        const f32x4 val = *reinterpret_cast<const f32x4*>(stg + row * TW_SP + sl * 16);
        if (col * TW_PX + row < HW) *reinterpret_cast<f32x4*>(ybase + (size_t)o * frame_y + (size_t)row * 64 + sl * 8) = val;
      }
      wave_sync();
    }
  };

  // step i: input frame u = ta - 1 + i in ring slot i % 3; accumulator slots: y[u - 1] in (i + 2) % 3
  // (complete after this step, stored), y[u] in i % 3, y[u + 1] in (i + 1) % 3
  tw_unroll(std::make_integer_sequence<int, NI>{}, [&](auto ic) __attribute__((always_inline)) {
    constexpr int I = decltype(ic)::value;
    constexpr int SX = I % NR, SP = (I + 2) % 3, SC = I % 3, SN = (I + 1) % 3;
    const int u = ta - 1 + I;
    if constexpr (I + PD < NI) load_frame(u + PD, xr[(I + PD) % NR]);  // PD frames ahead
    if constexpr (I >= 1 && I <= TS) load_res(u, rvq[I % 2]);       // stored at step I + 1
    if (u >= 0 && u < T) {
      // contributions: tap 2 -> y[u - 1] (if u - 1 >= ta), tap 1 -> y[u] (if u < ta + TS), tap 0 -> y[u + 1]
      // (if u + 1 < ta + TS); the conditions are compile-time in I (ta is the segment start)
      constexpr bool T2 = I >= 2, T1 = I >= 1 && I <= TS, T0 = I <= TS - 1;
#pragma unroll
      for (int s = 0; s < CS; ++s) {
        const bf16x8 b = xr[SX][s];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          if constexpr (KO & 4) {
            acc[SC][rb][0] += (float)b[rb] * (float)wfrag(1, s, rb)[0];
            continue;
          }
          if constexpr (T2) acc[SP][rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfrag(2, s, rb), b, acc[SP][rb], 0, 0, 0);
          if constexpr (T1) acc[SC][rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfrag(1, s, rb), b, acc[SC][rb], 0, 0, 0);
          if constexpr (T0) acc[SN][rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfrag(0, s, rb), b, acc[SN][rb], 0, 0, 0);
        }
      }
    }
    if constexpr (I >= 2) store_out(u - 1, acc[SP], rvq[(I - 1) % 2]);  // y[u - 1] = y[ta + I - 2], I - 2 in [0, TS)
  });
}

}  // namespace

bool twalk_bf16_supported(const ConvParams& p) {
  if (!p.in_bf16 || !p.out_bf16 || p.stem || p.x2 || !p.bias || p.x_c8 || p.y_c8) return false;
  if (!(p.KT == 3 && p.KH == 1 && p.KW == 1 && p.st == 1 && p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 0 && p.pw == 0))
    return false;
  if (p.Cout != 64 || !(p.Cin == 160 || p.Cin == 64) || p.Kp != 3 * p.Cin) return false;
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi || p.Ti % 8) return false;
  if ((size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin >= ((size_t)1 << 31)) return false;
  return true;
}

namespace {
template <int CS, int TS, int EF, int PD = 2, int W = 1, int KO = 0>
hipError_t launch_tw_e(const ConvParams& p, hipStream_t s) {
  const int HW = p.Hi * p.Wi;
  const int n_cols = (HW + TW_PX - 1) / TW_PX, n_seg = p.Ti / TS;
  const long waves = (long)p.N * n_cols * n_seg;
  const size_t lds = 64 * tw_pitch(16 * CS) + 64 * 4 + 4 * 32 * TW_SP;
  hipLaunchKernelGGL((conv_twalk_bf16<CS, TS, EF, PD, W, KO>), dim3((unsigned)((waves + 3) / 4)), dim3(256), lds, s, p,
                     n_cols, n_seg);
  return hipGetLastError();
}
template <int CS, int TS>
hipError_t launch_tw_t(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 0: return launch_tw_e<CS, TS, 0>(p, s);
    case 1: return launch_tw_e<CS, TS, 1>(p, s);
    case 2: return launch_tw_e<CS, TS, 2>(p, s);
    default: return launch_tw_e<CS, TS, 3>(p, s);
  }
}
template <int CS>
hipError_t launch_tw_c(const ConvParams& p, hipStream_t s) {
  // 16-frame segments where T allows (32-frame clips: 2 per clip column, 2 of 18 input frames re-read)
  return p.Ti % 16 == 0 ? launch_tw_t<CS, 16>(p, s) : launch_tw_t<CS, 8>(p, s);
}
}  // namespace

hipError_t launch_twalk_bf16(const ConvParams& p, hipStream_t s) {
  if (!twalk_bf16_supported(p)) return hipErrorInvalidValue;
  return p.Cin == 160 ? launch_tw_c<10>(p, s) : launch_tw_c<4>(p, s);
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench (tpp, ko 990 + v): v = 10 * PD + W, e.g. 21 = the first form (2 frames ahead, one
// wave per SIMD); TS 16 and the residual / ReLU flags of p
hipError_t launch_twalk_bf16_ko(const ConvParams& p, hipStream_t s, int v) {
  if (!twalk_bf16_supported(p) || p.Ti % 16) return hipErrorInvalidValue;
  const int ef = (p.res ? 1 : 0) | (p.relu ? 2 : 0);
  auto go = [&](auto cs) -> hipError_t {
    constexpr int CS = decltype(cs)::value;
    auto e = [&](auto efc) -> hipError_t {
      constexpr int EF = decltype(efc)::value;
      switch (v) {
        case 102: return launch_tw_e<CS, 16, EF, 2, 1, 1>(p, s);  // no stores
        case 103: return launch_tw_e<CS, 16, EF, 2, 1, 2>(p, s);  // no input loads
        case 104: return launch_tw_e<CS, 16, EF, 2, 1, 4>(p, s);  // no MFMAs
        case 21: return launch_tw_e<CS, 16, EF, 2, 1>(p, s);
        case 31: return launch_tw_e<CS, 16, EF, 3, 1>(p, s);
        case 41: return launch_tw_e<CS, 16, EF, 4, 1>(p, s);
        case 22: return launch_tw_e<CS, 16, EF, 2, 2>(p, s);
        case 32: if constexpr (CS <= 4) return launch_tw_e<CS, 16, EF, 3, 2>(p, s); break;
        case 42: if constexpr (CS <= 4) return launch_tw_e<CS, 16, EF, 4, 2>(p, s); break;
      }
      return hipErrorInvalidValue;
    };
    switch (ef) {
      case 0: return e(std::integral_constant<int, 0>{});
      case 1: return e(std::integral_constant<int, 1>{});
      case 2: return e(std::integral_constant<int, 2>{});
      default: return e(std::integral_constant<int, 3>{});
    }
  };
  return p.Cin == 160 ? go(std::integral_constant<int, 10>{}) : go(std::integral_constant<int, 4>{});
}
#endif
