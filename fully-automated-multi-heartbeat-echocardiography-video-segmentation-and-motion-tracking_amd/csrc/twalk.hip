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
#include <string.h>

#include <utility>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int tw_u32x4 __attribute__((ext_vector_type(4)));

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
// bit 1 ReLU, PD = input frames loaded ahead (register ring of PD + 1 frames), W = waves per SIMD,
// HV = 64-channel output halves (Cout = 64 HV; HV = 2: layer2's 128 channels, each block one half, the
// two halves of a column on one XCD so the second reads the input frames from its L2)
// KO (convbench knock-outs, wrong results): 1 no output stores, 2 no input loads in the walk, 4 no MFMAs
constexpr int TW_SP = 144;  // staging row pitch (bytes): 128 + 16, conflict-free 8-B accesses of 32 rows
template <int CS, int TS, int EF, int PD, int W, int KO = 0, int HV = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) void conv_twalk_bf16(ConvParams p, int n_cols,
                                                                                                   int n_seg) {
  constexpr int CIN = 16 * CS, KP = 3 * CIN, PITCH = tw_pitch(CIN);
  constexpr int NI = TS + 2;  // input frames per segment (one halo frame each side)
  extern __shared__ __align__(16) char smem[];  // [64 rows][PITCH] weights, 64 fp32 biases, staging
  float* sbias = reinterpret_cast<float*>(smem + 64 * PITCH);
  char* stg = smem + 64 * PITCH + 256 + (threadIdx.x >> 6) * 32 * TW_SP;  // this wave's staging rows

  const int tid = threadIdx.x, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  // HV = 2: blocks 16 j + x (half 0) and 16 j + 8 + x (half 1) hold the same columns and run on XCD x
  const int half = HV == 2 ? (blockIdx.x >> 3) & 1 : 0;
  const int bpair = HV == 2 ? (blockIdx.x >> 4) * 8 + (blockIdx.x & 7) : blockIdx.x;
  // weights -> LDS once per block (16-B chunks, row pitch PITCH): rows 64 half .. + 63
  {
    const char* w = reinterpret_cast<const char*>(p.w) + (size_t)64 * half * KP * 2;
    constexpr int CPR = KP * 2 / 16;  // 16-B chunks per weight row
    for (int c = tid; c < 64 * CPR; c += 256) {
      const int row = c / CPR, k = c - row * CPR;
      *reinterpret_cast<f32x4*>(smem + row * PITCH + k * 16) =
          *reinterpret_cast<const f32x4*>(w + ((size_t)row * KP) * 2 + k * 16);
    }
    if (tid < 64) sbias[tid] = p.bias[64 * half + tid];
  }
  __syncthreads();

  // this wave's (clip, 32-pixel column, frame segment)
  const int HW = p.Hi * p.Wi, T = p.Ti;
  int item = __builtin_amdgcn_readfirstlane(bpair * 4 + (tid >> 6));  // wave-uniform: scalar
  const int seg = item % n_seg;
  item /= n_seg;
  const int col = item % n_cols, clip = item / n_cols;
  if (clip >= p.N) return;  // (the grid is whole blocks of 4 waves; no barrier follows)
  const int ta = seg * TS;
  const int px = col * TW_PX + r;
  const bool pv = px < HW;  // lanes past the map load pixel 0 (their outputs are not stored)
  const __bf16* x = reinterpret_cast<const __bf16*>(p.x) + ((size_t)clip * T * HW + (pv ? px : 0)) * CIN + 8 * h;
  const size_t frame_x = (size_t)HW * CIN;
  // the column's pixel 0 (this half's channel 0) in the output and the residual
  constexpr int CO = 64 * HV;  // output channels = output pixel pitch (elements)
  __bf16* ybase = reinterpret_cast<__bf16*>(p.y) + ((size_t)clip * T * HW + col * TW_PX) * CO + 64 * half;
  const __bf16* rbase = reinterpret_cast<const __bf16*>(p.res) + ((size_t)clip * T * HW + col * TW_PX) * CO + 64 * half;
  const size_t frame_y = (size_t)HW * CO;

  constexpr int NR = PD + 1;
  bf16x8 xr[NR][CS];  // register ring: input frame ta - 1 + i in slot i % NR
  f32x16 acc[3][2];  // rolling outputs: y[u - 1], y[u], y[u + 1] of input frame u in slots (i+2)%3, i%3... (below)
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  // Every load is issued on every path -- a frame outside the clip (zero padding) reads the clip's end
  // frame and is zeroed before use (segment end steps only) -- so each wait counts exactly the memory
  // operations issued after the ones it needs (a conditional load made the compiler wait for the next
  // frame's loads too: vmcnt(9) .. vmcnt(5) in every step).
  auto load_frame = [&](int u, bf16x8 (&dst)[CS]) __attribute__((always_inline)) {
    if ((KO & 2) && u > ta + 1) return;
    const int uc = u < 0 ? 0 : u >= T ? T - 1 : u;
    const __bf16* src = x + (size_t)uc * frame_x;
#pragma unroll
    for (int s = 0; s < CS; ++s) dst[s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
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
  // Rows past the map: buffer resources over the column's valid rows (reads return zeros, stores are
  // dropped), no per-lane branches.
  f32x4 rvq[2][4];
  const int col_bytes = (HW - col * TW_PX < TW_PX ? HW - col * TW_PX : TW_PX) * 2 * CO;
  const int row_off = (lane >> 3) * 2 * CO + (lane & 7) * 16;
  auto load_res = [&](int o, f32x4 (&rq)[4]) __attribute__((always_inline)) {
    if constexpr (EF & 1) {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<__bf16*>(rbase + (size_t)o * frame_y), (short)0, col_bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        rq[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, row_off + k * 16 * CO, 0, 0));
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
      const __amdgpu_buffer_rsrc_t yr =
          __builtin_amdgcn_make_buffer_rsrc(ybase + (size_t)o * frame_y, (short)0, col_bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = 8 * k + (lane >> 3), sl = lane & 7;
        const f32x4 val = *reinterpret_cast<const f32x4*>(stg + row * TW_SP + sl * 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tw_u32x4, val), yr, row_off + k * 16 * CO, 0, 0);
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
    // only a segment's end steps can fall outside the clip: their frame is zeroed by a select (no branch)
    constexpr bool EDGE = I == 0 || I == NI - 1;
    const bool fv = u >= 0 && u < T;
    {
      // contributions: tap 2 -> y[u - 1] (if u - 1 >= ta), tap 1 -> y[u] (if u < ta + TS), tap 0 -> y[u + 1]
      // (if u + 1 < ta + TS); the conditions are compile-time in I (ta is the segment start)
      constexpr bool T2 = I >= 2, T1 = I >= 1 && I <= TS, T0 = I <= TS - 1;
#pragma unroll
      for (int s = 0; s < CS; ++s) {
        bf16x8 b = xr[SX][s];
        if constexpr (EDGE) b = fv ? b : bf16x8{};
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
  if (p.Kp != 3 * p.Cin) return false;
  // 64 output channels: the stem's and layer1's (Cin 64, 160). convbench builds also take layer2's 128
  // (Cin 256, 288; two 64-channel halves per column): measured and not taken by the product -- 0.138 /
  // 0.116 ms vs conv_patch_bf16's 0.110 / 0.096 without the residual, 0.145 / 0.126 vs 0.153 / 0.141 with
  // it (8-frame segments; profiles/r06l_twalk_layer2.txt)
#ifdef CLASFV_KNOCKOUTS
  if (!((p.Cout == 64 && (p.Cin == 160 || p.Cin == 64)) || (p.Cout == 128 && (p.Cin == 256 || p.Cin == 288))))
    return false;
#else
  if (!(p.Cout == 64 && (p.Cin == 160 || p.Cin == 64))) return false;
#endif
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi || p.Ti % 8) return false;
  if ((size_t)p.N * p.Ti * p.Hi * p.Wi * (p.Cin > p.Cout ? p.Cin : p.Cout) >= ((size_t)1 << 31)) return false;
  return true;
}

namespace {
template <int CS, int TS, int EF, int PD = 2, int W = 1, int KO = 0, int HV = 1>
hipError_t launch_tw_e(const ConvParams& p, hipStream_t s) {
  const int HW = p.Hi * p.Wi;
  const int n_cols = (HW + TW_PX - 1) / TW_PX, n_seg = p.Ti / TS;
  const long waves = (long)p.N * n_cols * n_seg;
  const size_t lds = 64 * tw_pitch(16 * CS) + 64 * 4 + 4 * 32 * TW_SP;
  const long blocks = (waves + 3) / 4;  // per half; HV = 2: 16 blocks per 8 block pairs
  hipLaunchKernelGGL((conv_twalk_bf16<CS, TS, EF, PD, W, KO, HV>), dim3((unsigned)(HV == 2 ? (blocks + 7) / 8 * 16 : blocks)),
                     dim3(256), lds, s, p, n_cols, n_seg);
  return hipGetLastError();
}
template <int CS, int TS, int HV>
hipError_t launch_tw_t(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 0: return launch_tw_e<CS, TS, 0, 2, 1, 0, HV>(p, s);
    case 1: return launch_tw_e<CS, TS, 1, 2, 1, 0, HV>(p, s);
    case 2: return launch_tw_e<CS, TS, 2, 2, 1, 0, HV>(p, s);
    default: return launch_tw_e<CS, TS, 3, 2, 1, 0, HV>(p, s);
  }
}
template <int CS, int HV = 1>
hipError_t launch_tw_c(const ConvParams& p, hipStream_t s) {
  // 16-frame segments where T allows (32-frame clips: 2 per clip column, 2 of 18 input frames re-read)
  return p.Ti % 16 == 0 ? launch_tw_t<CS, 16, HV>(p, s) : launch_tw_t<CS, 8, HV>(p, s);
}
}  // namespace

hipError_t launch_twalk_bf16(const ConvParams& p, hipStream_t s) {
  if (!twalk_bf16_supported(p)) return hipErrorInvalidValue;
#ifdef CLASFV_KNOCKOUTS
  if (p.Cout == 128) return p.Cin == 288 ? launch_tw_c<18, 2>(p, s) : launch_tw_c<16, 2>(p, s);
#endif
  return p.Cin == 160 ? launch_tw_c<10>(p, s) : launch_tw_c<4>(p, s);
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench (tpp, ko 990 + v): v = 10 * PD + W, e.g. 21 = the first form (2 frames ahead, one
// wave per SIMD); TS 16 and the residual / ReLU flags of p
hipError_t launch_twalk_bf16_ko(const ConvParams& p, hipStream_t s, int v) {
  if (!twalk_bf16_supported(p)) return hipErrorInvalidValue;
  const int ef = (p.res ? 1 : 0) | (p.relu ? 2 : 0);
  if (p.Cout == 128) {  // layer2 (two halves): v = 1000 PD + TS, e.g. 2016 = PD 2, TS 16
    auto g2 = [&](auto cs) -> hipError_t {
      constexpr int CS = decltype(cs)::value;
      auto e = [&](auto efc) -> hipError_t {
        constexpr int EF = decltype(efc)::value;
        switch (v) {
          case 1016: return p.Ti % 16 ? hipErrorInvalidValue : launch_tw_e<CS, 16, EF, 1, 1, 0, 2>(p, s);
          case 2016: return p.Ti % 16 ? hipErrorInvalidValue : launch_tw_e<CS, 16, EF, 2, 1, 0, 2>(p, s);
          case 1008: return launch_tw_e<CS, 8, EF, 1, 1, 0, 2>(p, s);
          case 2008: return launch_tw_e<CS, 8, EF, 2, 1, 0, 2>(p, s);
        }
        return hipErrorInvalidValue;
      };
      return ef == 3 ? e(std::integral_constant<int, 3>{}) : e(std::integral_constant<int, 2>{});
    };
    if (!p.relu) return hipErrorInvalidValue;
    return p.Cin == 288 ? g2(std::integral_constant<int, 18>{}) : g2(std::integral_constant<int, 16>{});
  }
  if (p.Ti % 16) return hipErrorInvalidValue;
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

#ifdef CLASFV_KNOCKOUTS
// ---------------------------------------------------------------------------------------------
// conv_twalk_x3 (round 6): the fp32 engines' stride-1 temporal 3x1x1 convs with 64 output channels as
// conv_twalk_bf16's frame walk on split-bf16 MFMAs: x = hi + mid + lo (each the bf16 of the remainder,
// fp32's 24 bits), the six products lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi (smallest first)
// accumulated in fp32, conv_dma_x3's arithmetic: fp32-accurate. conv_winot5 runs these as a Winograd
// F(4,3) on f32 MFMAs: 1.5 f32 products per output and channel pair = 24 bf16-product times; the split
// direct form needs 3 taps x 6 = 18, and walking frames reads every input frame once. Measured
// (profiles/r06h_twalk_x3.txt) and NOT in the product -- convbench builds only (CLASFV_KNOCKOUTS):
// layer1's 144 -> 64 0.886 ms vs conv_winot5's 0.856 (62 % MFMA-busy: the issue port is shared with
// 4 VALU per MFMA of splitting and epilogue work); the stem's 48 -> 64 0.332 vs 0.403 in convbench but
// 0.322 vs 0.333 inside the engine's forward (fp32 bench A/B 1414.2 / 1418.9 vs 1414.9 / 1417.0
// clips/s: a wash, so the engine keeps conv_winot5 for both).
//  * a wave owns 32 pixels x 32 output channels (one 32-row block) of a 16-frame segment; the two
//    channel halves of a column are blocks on one XCD (the second reads the input frames from its L2:
//    fetch 1.79 GB for 1.73 GB of input, 3.6 GB with the halves on different XCDs); weights of the
//    half -- 3 pieces x 32 rows x 3 Cin -- in LDS; two waves per SIMD (8-wave blocks);
//  * the input is read as fp32 straight into registers (channels-last, or the producer's 8-channel-
//    blocked layout, where a lane's 8 channels of one pixel are 32 contiguous bytes and 32 pixels one
//    1-KiB run), split into the three bf16 pieces once per frame and 16-channel step -- each piece feeds
//    3 taps -- and refilled with the next frame's step right after;
//  * no load or store is conditional (clamped end frames, zeroed by a multiply; buffer-resource rows),
//    so every wait counts exactly the memory operations issued after the one it needs;
//  * outputs (and a residual's rows) through per-wave LDS staging rows, whole 128-B half-pixel rows
//    per store instruction.
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int TX_SP = 144;  // staging row pitch: 32 fp32 channels (128 B) + 16

__host__ __device__ constexpr int tx_pitch(int cin) {  // bytes per weight row (3 cin bf16), odd 16-B count
  return (6 * cin / 16) % 2 == 0 ? 6 * cin + 16 : 6 * cin;
}

__device__ inline bf16x8 tx_pack(f32x4 a, f32x4 b) {
  return bf16x8{(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3], (__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
}

// CS = Cin / 16, TS = frames per segment, EF bit 0 residual, bit 1 ReLU, XC8: 8-channel-blocked input,
// W waves per SIMD (blocks of 4 W waves, one channel half)
template <int CS, int TS, int EF, bool XC8, int W>
__global__ __launch_bounds__(256 * W) __attribute__((amdgpu_waves_per_eu(W, W))) void conv_twalk_x3(ConvParams p, int n_cols,
                                                                                                     int n_seg) {
  constexpr int CIN = 16 * CS, KP = 3 * CIN, PITCH = tx_pitch(CIN), PIECE = 32 * PITCH;
  constexpr int NI = TS + 2;
  extern __shared__ __align__(16) char smem[];  // [3 pieces][32 rows][PITCH], 32 biases, staging
  float* sbias = reinterpret_cast<float*>(smem + 3 * PIECE);
  char* stg = smem + 3 * PIECE + 128 + (threadIdx.x >> 6) * 32 * TX_SP;

  const int tid = threadIdx.x, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  // the two channel halves of a block of columns run on one XCD (blocks are dispatched round-robin over
  // the 8 XCDs): the second reads the input frames from that XCD's L2 instead of HBM
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int half = slot & 1;  // output channels 32 half .. + 31
  const int pair = (slot >> 1) * 8 + xcd;
  {
    // p.w: the pieces' images [3][Cout][KP] bf16 (twalk_x3_weight_image); this half's 32 rows
    const char* w = reinterpret_cast<const char*>(p.w);
    constexpr int CPR = KP * 2 / 16;
    for (int c = tid; c < 3 * 32 * CPR; c += 256 * W) {
      const int pr = c / CPR, k = c - pr * CPR, pc = pr >> 5, row = pr & 31;
      *reinterpret_cast<f32x4*>(smem + pc * PIECE + row * PITCH + k * 16) =
          *reinterpret_cast<const f32x4*>(w + (((size_t)pc * 64 + 32 * half + row) * KP) * 2 + k * 16);
    }
    if (tid < 32) sbias[tid] = p.bias[32 * half + tid];
  }
  __syncthreads();

  const int HW = p.Hi * p.Wi, T = p.Ti;
  int item = __builtin_amdgcn_readfirstlane(pair * 4 * W + (tid >> 6));  // wave-uniform: scalar
  const int seg = item % n_seg;
  item /= n_seg;
  const int col = item % n_cols, clip = item / n_cols;
  if (clip >= p.N) return;  // (no barrier follows)
  const int ta = seg * TS;
  const int px = col * 32 + r;
  const bool pv = px < HW;
  const size_t mtot = (size_t)p.N * T * HW;  // voxels of the whole input (8-channel-blocked plane size)
  const size_t vox0 = (size_t)clip * T * HW + (pv ? px : 0);
  const float* xf = reinterpret_cast<const float*>(p.x);
  float* ybase = reinterpret_cast<float*>(p.y) + ((size_t)clip * T * HW + col * 32) * 64 + 32 * half;
  const float* rbase = reinterpret_cast<const float*>(p.res) + ((size_t)clip * T * HW + col * 32) * 64 + 32 * half;
  const size_t frame_y = (size_t)HW * 64;

  // lane (r, h): pixel r, channels 16 s + 8 h .. + 7 of each 16-channel step s; one frame, each step's
  // registers refilled with the next frame's as soon as they are split (a whole frame step of lead)
  f32x4 xr[CS][2];
  f32x16 ac16[3];  // rolling outputs (channel 8 g + 4 h + e of pixel r in register 4 g + e)
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) ac16[a][e] = 0.f;

  // per-lane base (pixel, channel half) + wave-uniform frame / channel-step offsets
  const float* xlane = XC8 ? xf + ((size_t)h * mtot + vox0) * 8 : xf + vox0 * CIN + 8 * h;
  // every load is issued on every path (frames past the clip ends read the end frame, unused), so the
  // wait for a step's registers counts exactly the loads issued after them
  auto load_step = [&](int u, int s, f32x4 (&dst)[2]) __attribute__((always_inline)) {
    const int uc = u < 0 ? 0 : u >= T ? T - 1 : u;
    const size_t off = XC8 ? ((size_t)(2 * s) * mtot + (size_t)uc * HW) * 8 : (size_t)uc * HW * CIN + 16 * s;
    const float* src = xlane + off;
    dst[0] = *reinterpret_cast<const f32x4*>(src);
    dst[1] = *reinterpret_cast<const f32x4*>(src + 4);
  };
  const char* wa = smem + r * PITCH + (8 * h) * 2;
  auto wfrag = [&](int pc, int kt, int s) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8*>(wa + pc * PIECE + (kt * CIN + 16 * s) * 2);
  };
#pragma unroll
  for (int s = 0; s < CS; ++s) load_step(ta - 1, s, xr[s]);
  // weight fragments [piece][tap] of one 16-channel step; at one wave per SIMD read one step ahead
  // (double-buffered), at two the partner wave hides their latency
  constexpr int NWB = W == 1 ? 2 : 1;
  bf16x8 wq[NWB][3][3];
  auto load_w = [&](int s, bf16x8 (&d)[3][3]) __attribute__((always_inline)) {
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
#pragma unroll
      for (int kt = 0; kt < 3; ++kt) d[pc][kt] = wfrag(pc, kt, s);
  };
  if constexpr (NWB == 2) load_w(0, wq[0]);

  // output / residual rows: store instruction k moves rows 8 k .. 8 k + 7 (lane: row 8 k + lane / 8,
  // 16-B slot lane % 8 of the 128-B half-pixel row); at one wave per SIMD the residual of an epilogue is
  // loaded one step ahead in that layout (double-buffered), at two in the epilogue
  constexpr int NRB = W == 1 ? 2 : 1;
  f32x4 rvq[NRB][4];
  // residual / output rows through buffer resources over the frame's 32-pixel column (rows past the
  // map read zeros / are dropped): no per-lane branches, so no load or store is conditional either
  const int col_bytes = (HW - col * 32 < 32 ? HW - col * 32 : 32) * 256;
  const int row_off = (lane >> 3) * 256 + (lane & 7) * 16;
  auto load_res = [&](int o, f32x4 (&rq)[4]) __attribute__((always_inline)) {
    if constexpr (EF & 1) {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(rbase + (size_t)o * frame_y), (short)0, col_bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        rq[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, row_off + k * 2048, 0, 0));
    }
  };
  auto wave_sync = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  };
  auto store_out = [&](int o, f32x16& ac, const f32x4 (&rq)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + 8 * g + 4 * h);
      const f32x4 v = {ac[4 * g] + bv[0], ac[4 * g + 1] + bv[1], ac[4 * g + 2] + bv[2], ac[4 * g + 3] + bv[3]};
      *reinterpret_cast<f32x4*>(stg + r * TX_SP + (8 * g + 4 * h) * 4) = v;
#pragma unroll
      for (int q = 0; q < 4; ++q) ac[4 * g + q] = 0.f;
    }
    wave_sync();
    const __amdgpu_buffer_rsrc_t yr =
        __builtin_amdgcn_make_buffer_rsrc(ybase + (size_t)o * frame_y, (short)0, col_bytes, 0x00020000);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 8 * k + (lane >> 3), sl = lane & 7;
      f32x4 val = *reinterpret_cast<const f32x4*>(stg + row * TX_SP + sl * 16);
      if constexpr (EF & 1) val += rq[k];
      if constexpr (EF & 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) val[q] = relu1(val[q]);
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), yr, row_off + k * 2048, 0, 0);
    }
    wave_sync();
  };

  tw_unroll(std::make_integer_sequence<int, NI>{}, [&](auto ic) __attribute__((always_inline)) {
    constexpr int I = decltype(ic)::value;
    constexpr int SP = (I + 2) % 3, SC = I % 3, SN = (I + 1) % 3;
    const int u = ta - 1 + I;
    if constexpr (W == 1 && I >= 1 && I <= TS) load_res(u, rvq[I % 2]);  // stored at step I + 1
    // only the segment's end steps can fall outside the clip: their frame is zeroed (a multiply, not
    // a branch, so the whole segment stays one basic block the scheduler interleaves across steps)
    constexpr bool EDGE = I == 0 || I == NI - 1;
    const float fm = u >= 0 && u < T ? 1.f : 0.f;
    constexpr bool T2 = I >= 2, T1 = I >= 1 && I <= TS, T0 = I <= TS - 1;
    tw_unroll(std::make_integer_sequence<int, CS>{}, [&](auto sc) __attribute__((always_inline)) {
      constexpr int S = decltype(sc)::value, B = NWB == 2 ? (I * CS + S) % 2 : 0;
      if constexpr (NWB == 1) load_w(S, wq[0]);
      else if constexpr (I * CS + S + 1 < NI * CS) load_w((S + 1) % CS, wq[1 - B]);
      bf16x8 xh, xm, xl;
      {
        f32x4 a = xr[S][0], b = xr[S][1];
        if constexpr (EDGE) a *= fm, b *= fm;
        xh = tx_pack(a, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] -= (float)xh[e], b[e] -= (float)xh[4 + e];
        xm = tx_pack(a, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] -= (float)xm[e], b[e] -= (float)xm[4 + e];
        xl = tx_pack(a, b);
      }
      if constexpr (I + 1 < NI) load_step(u + 1, S, xr[S]);
      {
        auto prod = [&](int kt, f32x16& c) __attribute__((always_inline)) {
          const bf16x8 wh = wq[B][0][kt], wm = wq[B][1][kt], wl = wq[B][2][kt];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, c, 0, 0, 0);
        };
        if constexpr (T2) prod(2, ac16[SP]);
        if constexpr (T1) prod(1, ac16[SC]);
        if constexpr (T0) prod(0, ac16[SN]);
      }
    });
    if constexpr (I >= 2) {
      if constexpr (W == 2) load_res(u - 1, rvq[0]);
      store_out(u - 1, ac16[SP], rvq[NRB == 2 ? (I - 1) % 2 : 0]);
    }
    __builtin_amdgcn_sched_barrier(0);  // one scheduling region per frame step
  });
}

}  // namespace

// conv_twalk_x3's weight pieces: [3][cout][kp] bf16, natural k order (k = tap cin + c), each the bf16
// (round to nearest) of the remainder in double, as dma_x3_weight_image's
void twalk_x3_weight_image(const float* w, int cout, int kp, uint16_t* out) {
  for (size_t i = 0; i < (size_t)cout * kp; ++i) {
    double rr = (double)w[i];
    for (int pc = 0; pc < 3; ++pc) {
      float f = (float)rr;
      uint32_t u;
      memcpy(&u, &f, 4);
      const uint16_t b = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
      const uint32_t ub = (uint32_t)b << 16;
      float fb;
      memcpy(&fb, &ub, 4);
      out[(size_t)pc * cout * kp + i] = b;
      rr -= fb;
    }
  }
}

bool twalk_x3_supported(const ConvParams& p) {
  // (ReLU: every 64-channel temporal conv of the encoder ends in one)
  if (p.in_bf16 || p.out_bf16 || p.stem || p.x2 || !p.bias || p.y_c8 || !p.relu) return false;
  if (!(p.KT == 3 && p.KH == 1 && p.KW == 1 && p.st == 1 && p.sh == 1 && p.sw == 1 && p.pt == 1 && p.ph == 0 && p.pw == 0))
    return false;
  if (p.Cout != 64 || p.Kp != 3 * p.Cin) return false;
  if (!(p.Cin == 144 || p.Cin == 48)) return false;
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi || p.Ti % 8) return false;
  if ((size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin >= ((size_t)1 << 31)) return false;
  return true;
}

namespace {
template <int CS, int TS, int EF, bool XC8, int W>
hipError_t launch_tx_e(const ConvParams& p, hipStream_t s) {
  const int HW = p.Hi * p.Wi;
  const int n_cols = (HW + 31) / 32, n_seg = p.Ti / TS;
  const long waves = (long)p.N * n_cols * n_seg;
  const size_t lds = 3 * 32 * tx_pitch(16 * CS) + 128 + 4 * W * 32 * TX_SP;
  const long pairs = (waves + 4 * W - 1) / (4 * W);  // blocks per channel half; 16 blocks per 8 pairs
  hipLaunchKernelGGL((conv_twalk_x3<CS, TS, EF, XC8, W>), dim3((unsigned)((pairs + 7) / 8 * 16)), dim3(256 * W), lds, s, p,
                     n_cols, n_seg);
  return hipGetLastError();
}
template <int CS, int TS, bool XC8, int W>
hipError_t launch_tx_t(const ConvParams& p, hipStream_t s) {
  return p.res ? launch_tx_e<CS, TS, 3, XC8, W>(p, s) : launch_tx_e<CS, TS, 2, XC8, W>(p, s);
}
template <int CS, int W>
hipError_t launch_tx_c(const ConvParams& p, hipStream_t s) {
  if (p.x_c8) return p.Ti % 16 == 0 ? launch_tx_t<CS, 16, true, W>(p, s) : launch_tx_t<CS, 8, true, W>(p, s);
  return p.Ti % 16 == 0 ? launch_tx_t<CS, 16, false, W>(p, s) : launch_tx_t<CS, 8, false, W>(p, s);
}
}  // namespace

// p.w: twalk_x3_weight_image of the conv's folded weights
hipError_t launch_twalk_x3(const ConvParams& p, hipStream_t s) {
  if (!twalk_x3_supported(p)) return hipErrorInvalidValue;
  return p.Cin == 144 ? launch_tx_c<9, 2>(p, s) : launch_tx_c<3, 2>(p, s);
}

// v = waves per SIMD (1, 2)
hipError_t launch_twalk_x3_ko(const ConvParams& p, hipStream_t s, int v) {
  if (!twalk_x3_supported(p)) return hipErrorInvalidValue;
  if (v == 1) return p.Cin == 144 ? launch_tx_c<9, 1>(p, s) : launch_tx_c<3, 1>(p, s);
  return p.Cin == 144 ? launch_tx_c<9, 2>(p, s) : launch_tx_c<3, 2>(p, s);
}
#endif  // CLASFV_KNOCKOUTS
