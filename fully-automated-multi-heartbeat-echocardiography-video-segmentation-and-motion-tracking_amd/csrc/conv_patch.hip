// Patch-staged bf16 implicit GEMM for the stride-1 convs of the R(2+1)D-18 encoder in bf16
// (BASELINE config[4]: bf16 activations/weights, fp32 accumulation): the Conv2Plus1D spatial 1x3x3
// and temporal 3x1x1 halves (torchvision Conv2Plus1D, called from
// src/model/R2plus1D_18_MotionNet.py:29-37) and the stem's temporal 3x1x1 conv.
//
// Why: conv_dma (conv.hip) gathers the im2col A tile straight from global memory, so every input
// voxel crosses the L2 -> LDS path once per tap; in bf16 the MFMAs are 16x faster than in fp32 and
// that gather, not the matrix cores, sets the time. Here a block's output tile is 4 frames x 64
// pixels (8x8 for the spatial conv, 64 consecutive pixels of the flattened map for the temporal
// one) x 16*NT output channels; for each 32-channel chunk the input patch it needs (4 x 10 x 10 or
// 6 x 64 pixels x 64 B) is copied to LDS once and every tap reads its A fragments from it at a
// pixel offset: 9 x 256 (3 x 256) gathered rows become 400 (384).
//  * wave w owns output frame t0 + w: 4 m tiles (64 voxels) x NT n tiles (up to 160 channels), so
//    per 32-deep K step a wave issues 4*NT MFMAs (v_mfma_f32_16x16x32_bf16) on 4 + NT LDS reads,
//    with one block barrier per step;
//  * K order: chunk-major, tap-minor (step s = TAPS*chunk + tap); weights keep conv_dma's image
//    [Cout_alloc][Kp] with k = tap*Cin + c, so one B row segment is w[n][tap*Cin + 32*chunk ..];
//  * patch image: double-buffered, pixel rows of 64 B, 16-B slot q of pixel p stored at
//    q ^ g[(p >> 2) & 3]; B ring: 3 stages of NT x 16 rows x 64 B, one per step. At NT = 10 the
//    spatial kernel's LDS is exactly 80 KiB: two blocks (8 waves) per CU;
//  * all copies are LDS-DMA (global_load_lds_dwordx4), 1-KiB pieces dealt round-robin to the
//    waves (piece j to wave j % 4, no sink slots); counted vmcnt with per-wave immediates: at step
//    s a wave waits for its own share of B(s) (and, by in-order completion, of the chunk's patch),
//    then a block barrier; the next chunk's patch is issued at the chunk's tap 0;
//  * epilogue: the MFMAs compute D^T = W . A^T, so a lane holds 4 consecutive output channels of
//    one voxel: folded-BN bias, optional residual, ReLU, 8-B bf16 stores; voxels outside the map
//    (ragged 28/14/7-pixel maps, partial pixel tiles) are masked.
#include <hip/hip_bf16.h>
#include <stdlib.h>

#include <utility>

#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// slot swizzle g = {0, 2, 3, 1} as arithmetic: a runtime-indexed constant array is a global load,
// and its in-order vmcnt wait would drain the whole DMA ring in front of every A read
__device__ inline int gsw(int i) { return (0x78 >> (2 * i)) & 3; }

__device__ inline int xcd_swizzle_p(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Patch geometry: KT = 1 -> 1x3x3 conv on 8x8-pixel tiles, KT = 3 -> 3x1x1 conv on 64 pixels;
// FR output frames per block.
template <int KT, int FR>
struct PGeo {
  static constexpr bool SPATIAL = KT == 1;
  static constexpr int TAPS = SPATIAL ? 9 : 3;
  static constexpr int MT = FR;                              // m tiles (16 voxels) per wave
  static constexpr int PF = FR + KT - 1;                     // patch frames
  static constexpr int PR = SPATIAL ? 10 : 1, PC = SPATIAL ? 10 : 64;
  static constexpr int FPIX = PR * PC;                       // patch pixels per frame
  static constexpr int PPIX = PF * FPIX;
  static constexpr int PIECES = (PPIX + 15) / 16;            // 1-KiB DMA pieces (16 pixels x 64 B)
  static constexpr int BYTES = PIECES * 1024;
};

template <int V>
__device__ inline void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(V) : "memory");
}

// An epilogue's bias / residual load through a global-address-space (1) pointer: the compiler then knows
// it cannot alias the LDS staging rows written between the loads and issues them together -- through
// the generic pointer every load waited for the previous staging write: 64 serialized load -> vmcnt(0)
// round trips per wave in conv_patch_bf16's temporal epilogue.
template <class V, class T>
__device__ inline V gload(const T* p) {
  typedef const V __attribute__((address_space(1))) GV;
  return *(GV*)(const __attribute__((address_space(1))) void*)p;
}

// address (bytes) of one 16-B LDS-DMA source: uniform base + per-lane offset (the saddr form)
__device__ inline void dma16(const char* base, unsigned off, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off),
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
__device__ inline void dma16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <int... I, class F>
__device__ inline void for_taps(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

// S = B ring depth (B(s) is fetched S-1 steps ahead); OCC = blocks per CU (the LDS budget and the
// register cap follow from it).
// STG: LDS-staged output stores (the product form; false = 8-B stores from the accumulator layout,
// convbench A/B)
// EF: epilogue flags at compile time, bit 0 residual, bit 1 ReLU (runtime flags kept both forms of every
// epilogue statement in the code)
template <int NT, int KT, int FR, int S, int OCC, bool STG = true, int EF = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void conv_patch_bf16(
    ConvParams p, int n_tiles, int ptw, int npt, int t_tiles) {
  using G = PGeo<KT, FR>;
  constexpr int TAPS = G::TAPS, MT = G::MT;
  static_assert(S >= 2 && S <= TAPS + 1, "wait counts below assume S - 1 <= TAPS");
  constexpr int PW = (G::PIECES + 3) / 4, BW = (NT + 3) / 4;  // DMAs per wave (uniform counts)
  constexpr int B_STAGE = NT * 1024, B0 = 2 * G::BYTES, SINK = B0 + S * B_STAGE;
  constexpr int LDS = SINK + 1024;
  static_assert(OCC * LDS <= 160 * 1024, "LDS budget");
  __shared__ __align__(16) char smem[LDS];

  const __bf16* x = reinterpret_cast<const __bf16*>(p.x);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  int tile = xcd_swizzle_p(blockIdx.x, gridDim.x);
  const int n0 = (tile % n_tiles) * 16 * NT;
  tile /= n_tiles;
  const int pt = tile % npt;
  tile /= npt;
  const int t0 = (tile % t_tiles) * FR;
  const int clip = tile / t_tiles;
  const int HW = p.Hi * p.Wi;
  const int h0 = G::SPATIAL ? (pt / ptw) * 8 : 0, w0 = G::SPATIAL ? (pt % ptw) * 8 : 0;
  const int hw0 = G::SPATIAL ? 0 : pt * 64;
  const int Cin = p.Cin;

  // patch DMA: piece j = wid + 4*i writes pixels 16j .. 16j+15, lane -> pixel 16j + lane/4,
  // physical slot lane & 3 (fetches logical slot (lane & 3) ^ g); pieces past the patch land in
  // the sink, pixels outside the map read the zero block
  int pv[PW];
  unsigned psl[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int pix = (wid + 4 * i) * 16 + (lane >> 2);
    psl[i] = (unsigned)(((lane & 3) ^ gsw((pix >> 2) & 3)) * 16);
    pv[i] = -1;
    if (pix < G::PPIX) {
      const int f = pix / G::FPIX, r = pix - f * G::FPIX;
      if constexpr (G::SPATIAL) {
        const int pr = r / G::PC, pc = r - pr * G::PC;
        const int ti = t0 + f, hi = h0 - 1 + pr, wi = w0 - 1 + pc;
        if (ti < p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
          pv[i] = ((clip * p.Ti + ti) * p.Hi + hi) * p.Wi + wi;
      } else {
        const int ti = t0 - 1 + f, hw = hw0 + r;
        if ((unsigned)ti < (unsigned)p.Ti && hw < HW) pv[i] = (clip * p.Ti + ti) * HW + hw;
      }
    }
  }
  auto issue_patch = [&](int c, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wid + 4 * i;
      const void* src = pv[i] >= 0 ? (const void*)(reinterpret_cast<const char*>(x + (size_t)pv[i] * Cin + 32 * c) + psl[i])
                                   : p.zero;
      dma16(src, smem + (j < G::PIECES ? buf * G::BYTES + j * 1024 : SINK));
    }
  };
  // B DMA (conv_dma's swizzled 64-B rows): piece j = wid + 4*i is n tile j; per-lane byte offsets
  // from the block's weight rows, the step's K offset in the uniform base
  const char* wb = reinterpret_cast<const char*>(p.w) + (size_t)n0 * p.Kp * 2;
  unsigned boff[BW];
  {
    const int drow = lane >> 2, dq = (lane & 3) ^ gsw((drow >> 2) & 3);
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      boff[i] = (unsigned)(((j < NT ? j : 0) * 16 + drow) * p.Kp + 8 * dq) * 2u;
    }
  }
  const int nc = Cin / 32;
  // B(c, tap) -> ring slot (TAPS*c + tap) % S; chunks past the end re-read chunk 0 into a slot
  // nobody reads
  auto issue_b = [&](int c, int tap, int slot) __attribute__((always_inline)) {
    const char* base = wb + (size_t)(tap * Cin + 32 * (c < nc ? c : 0)) * 2;
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      dma16(base, boff[i], smem + (j < NT ? B0 + slot * B_STAGE + j * 1024 : SINK));
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragment i of this lane: block voxel m = 16*(MT*wid + i) + l16; LDS byte address of its
  // 16-B slot q at every tap (patch buffer 0)
  int aaddr[TAPS][MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = 16 * (MT * wid + i) + l16, f = m >> 6, px = m & 63;
    const int base = G::SPATIAL ? (f * G::PR + (px >> 3)) * G::PC + (px & 7) : f * 64 + px;
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int pix = base + (G::SPATIAL ? (tap / 3) * G::PC + tap % 3 : tap * 64);
      aaddr[tap][i] = pix * 64 + ((q ^ gsw((pix >> 2) & 3)) << 4);
    }
  }
  const int b_rd = B0 + l16 * 64 + (q ^ gsw(l16 >> 2)) * 16;

  issue_patch(0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k) issue_b(k / TAPS, k % TAPS, k);
  int slot = 0;  // ring slot of B(s) (wave-uniform)

  for (int c = 0; c < nc; ++c) {
    const bool more = c + 1 < nc;
    const int pbuf = (c & 1) * G::BYTES;
    for_taps(std::make_integer_sequence<int, TAPS>{}, [&](auto tc) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tc)::value;
      // B(s) landed; in flight may stay B(s+1) .. B(s+S-2) and, at taps 1 .. S-1, the next chunk's
      // patch (issued at tap 0 after B(s)). At tap 0 the chunk's own patch was issued TAPS steps
      // ago, before B(s) whenever S - 1 <= TAPS.
      if constexpr (TAP >= 1 && TAP <= S - 1) {
        if (more) vm_wait<(S - 2) * BW + PW>();
        else vm_wait<(S - 2) * BW>();
      } else {
        vm_wait<(S - 2) * BW>();
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      constexpr int T2 = (TAP + S - 1) % TAPS, C2 = (TAP + S - 1) / TAPS;
      const int slot_new = slot == 0 ? S - 1 : slot - 1;  // (s + S - 1) % S
      issue_b(c + C2, T2, slot_new);
      if constexpr (TAP == 0) {
        if (more) issue_patch(c + 1, (c + 1) & 1);
      }
      bf16x8 a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = *reinterpret_cast<const bf16x8*>(smem + pbuf + aaddr[TAP][i]);
      const char* bs = smem + b_rd + slot * B_STAGE;
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + j * 1024);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      slot = slot + 1 == S ? 0 : slot + 1;
    });
  }
  vm_wait<0>();  // the past-the-end B fetches land before the block's LDS is released

  // epilogue: acc[i][j] holds channels n0 + 16j + 4q .. +3 of block voxel 16*(MT*wid + i) + l16
  const __bf16* res = reinterpret_cast<const __bf16*>(p.res);
  __bf16* y = reinterpret_cast<__bf16*>(p.y);
  // global voxel index of block voxel m (false outside the map)
  auto voxel = [&](int m, size_t& gm) __attribute__((always_inline)) {
    const int f = m >> 6, px = m & 63, to = t0 + f;
    if constexpr (G::SPATIAL) {
      const int ho = h0 + (px >> 3), wo = w0 + (px & 7);
      gm = (((size_t)clip * p.To + to) * p.Ho + (ho < p.Ho ? ho : 0)) * p.Wo + (wo < p.Wo ? wo : 0);
      return to < p.To && ho < p.Ho && wo < p.Wo;
    } else {
      const int hw = hw0 + px;
      gm = ((size_t)clip * p.To + to) * HW + (hw < HW ? hw : 0);
      return to < p.To && hw < HW;
    }
  };
  // the block's bias values, one (wave-uniform) branch for all of them (a branch per load serialized
  // the epilogue's loads)
  f32x4 bv[NT];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < NT; ++j) bv[j] = gload<f32x4>(p.bias + n0 + j * 16 + 4 * q);
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto finish = [&](int i, int j, size_t gm) __attribute__((always_inline)) {
    const int n = n0 + j * 16 + 4 * q;
    f32x4 v = acc[i][j] + bv[j];
    if constexpr (EF & 1) {
      const bf16x4 r = gload<bf16x4>(res + gm * p.Cout + n);
      v += f32x4{(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
    }
    if constexpr (EF & 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = relu1(v[e]);
    }
    return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  };
  if constexpr (!STG) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      size_t gm;
      if (!voxel(16 * (MT * wid + i) + l16, gm)) continue;
#pragma unroll
      for (int j = 0; j < NT; ++j) *reinterpret_cast<bf16x4*>(y + gm * p.Cout + n0 + j * 16 + 4 * q) = finish(i, j, gm);
    }
  } else {
    // LDS-staged: a lane's 8-B pieces hit 16 voxels per store instruction (16 partial lines); staged
    // in the dead patch / weight buffers as [16 MT voxels][NT*32 B + 16] per wave, they leave as
    // MT*NT/2 16-B-per-lane stores of whole voxel segments (contiguous runs when the block covers
    // every channel). convbench: see profiles/r04_patch32_bf16.txt
    // MH m tiles per pass: all MT when the 4 waves' staging fits the block's LDS, else half
    constexpr int SEG = NT * 32, VS = SEG + 16;
    constexpr int MH = 4 * 16 * MT * VS <= LDS ? MT : MT / 2, INS = 16 * MH * SEG / 1024;
    static_assert(4 * 16 * MH * VS <= LDS, "staging fits the block's LDS");
    static_assert(16 * MH * SEG % 1024 == 0, "whole store instructions");
    char* st = smem + wid * 16 * MH * VS;
    __builtin_amdgcn_s_barrier();  // every wave is past its last patch / weight read
#pragma unroll
    for (int i0 = 0; i0 < MT; i0 += MH) {
#pragma unroll
      for (int i = i0; i < i0 + MH; ++i) {
        size_t gm = 0;
        if constexpr (EF & 1) voxel(16 * (MT * wid + i) + l16, gm);
#pragma unroll
        for (int j = 0; j < NT; ++j)
          *reinterpret_cast<bf16x4*>(st + (16 * (i - i0) + l16) * VS + (16 * j + 4 * q) * 2) = finish(i, j, gm);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      // the pass's 16 MH voxels: block voxel mp + v (v < 16 MH), frame f = mp >> 6 of the block, pixel
      // px0 + v of its 64 (spatial: rows px0 / 8 + v / 8 of the 8x8 tile, column v % 8); store
      // addresses = a wave-uniform base + a small per-lane offset, masks only on edge tiles
      const int mp = 16 * (MT * wid + i0), f = mp >> 6, px0 = mp & 63, to = t0 + f;
      __bf16* yb;
      bool full;
      int row_el = 0;
      if constexpr (G::SPATIAL) {
        yb = y + ((((size_t)clip * p.To + to) * p.Ho + h0 + px0 / 8) * p.Wo + w0) * p.Cout + n0;
        full = to < p.To && h0 + px0 / 8 + 2 * MH <= p.Ho && w0 + 8 <= p.Wo;
        row_el = p.Wo * p.Cout;
      } else {
        yb = y + (((size_t)clip * p.To + to) * HW + hw0 + px0) * p.Cout + n0;
        full = to < p.To && hw0 + px0 + 16 * MH <= HW;
      }
#pragma unroll
      for (int k = 0; k < INS; ++k) {
        const int e = 1024 * k + 16 * lane, v = e / SEG, off = e - v * SEG;
        const bf16x8 val = *reinterpret_cast<const bf16x8*>(st + v * VS + off);
        const int lo = G::SPATIAL ? (v >> 3) * row_el + (v & 7) * p.Cout + off / 2 : v * p.Cout + off / 2;
        bool ok = full;
        if (!full) {
          if constexpr (G::SPATIAL) ok = to < p.To && h0 + px0 / 8 + (v >> 3) < p.Ho && w0 + (v & 7) < p.Wo;
          else ok = to < p.To && hw0 + px0 + v < HW;
        }
        if (ok) {
          if constexpr (EF & 4) {
            __builtin_nontemporal_store(val, reinterpret_cast<bf16x8*>(yb + lo));
          } else {
            *reinterpret_cast<bf16x8*>(yb + lo) = val;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
  }
}

template <int NT, int KT, int FR, int S>
constexpr int patch_occ() {
  constexpr int lds = 2 * PGeo<KT, FR>::BYTES + S * NT * 1024 + 1024;
  constexpr int occ = 160 * 1024 / lds;
  return occ > 4 ? 4 : occ;
}

struct PatchGrid {
  int ptw, npt, tt;
  long base;  // blocks per n tile
};

PatchGrid patch_grid(const ConvParams& p, int fr) {
  PatchGrid g{};
  if (p.KT == 1) {
    g.ptw = (p.Wo + 7) / 8;
    g.npt = g.ptw * ((p.Ho + 7) / 8);
  } else {
    g.npt = (p.Ho * p.Wo + 63) / 64;
  }
  g.tt = (p.To + fr - 1) / fr;
  g.base = (long)p.N * g.tt * g.npt;
  return g;
}

template <int NT, int KT, int FR, int S, bool STG, int EF>
hipError_t launch_pe(const ConvParams& p, hipStream_t s) {
  const PatchGrid g = patch_grid(p, FR);
  const int n_tiles = p.Cout / (16 * NT);
  hipLaunchKernelGGL((conv_patch_bf16<NT, KT, FR, S, patch_occ<NT, KT, FR, S>(), STG, EF>), dim3((unsigned)(g.base * n_tiles)),
                     dim3(256), 0, s, p, n_tiles, g.ptw, g.npt, g.tt);
  return hipGetLastError();
}

template <int NT, int KT, int FR, int S = 3, bool STG = true>
hipError_t launch_p(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 0: return launch_pe<NT, KT, FR, S, STG, 0>(p, s);
    case 1: return launch_pe<NT, KT, FR, S, STG, 1>(p, s);
    case 2: return launch_pe<NT, KT, FR, S, STG, 2>(p, s);
    default: return launch_pe<NT, KT, FR, S, STG, 3>(p, s);
  }
}

// Output frames per block and B ring depth (tools/bench_patch.sh): 1x3x3 convs 2 frames, 2 stages
// (a 2-deep ring measured as fast as 3-5 stages and leaves the LDS for 3 blocks per CU at NT = 10);
// 3x1x1 convs 4 frames (the 6-frame patch halves the temporal halo's re-fetch against 2 frames), 3
// stages.
template <int KT>
constexpr int product_fr() {
  return KT == 1 ? 2 : 4;
}
template <int KT>
constexpr int product_s() {
  return KT == 1 ? 2 : 3;
}

template <int KT>
hipError_t launch_nt(const ConvParams& p, int nt, hipStream_t s) {
  constexpr int FR = product_fr<KT>(), S = product_s<KT>();
  switch (nt) {
    case 10: return launch_p<10, KT, FR, S>(p, s);
    case 9: return launch_p<9, KT, FR, S>(p, s);
    case 8: return launch_p<8, KT, FR, S>(p, s);
    case 6: return launch_p<6, KT, FR, S>(p, s);
    case 5: return launch_p<5, KT, FR, S>(p, s);
    case 4: return launch_p<4, KT, FR, S>(p, s);
  }
  return hipErrorInvalidValue;
}

// N tile: the widest (fewest A re-reads, most MFMAs per LDS read) that still gives about two
// blocks per CU; the narrowest legal one when none does (layer4's 7x7 maps). 3x1x1 convs take the
// wider tile from 448 blocks (profiles/r02h_convbench_patch_sweep.txt: layer3 temporal, 480 blocks
// at NT = 8 vs 960 at NT = 4: 0.061 vs 0.069 ms).
int patch_pick_nt(const ConvParams& p, int force_nt) {
  const int n16 = p.Cout / 16;
  const long base = patch_grid(p, p.KT == 1 ? product_fr<1>() : product_fr<3>()).base;
  const long enough = p.KT == 3 ? 448 : 512;
  int pick = 0;
  for (int nt : {10, 9, 8, 6, 5, 4}) {
    if (n16 % nt) continue;
    if (force_nt > 0) {
      if (nt == force_nt) return nt;
      continue;
    }
    pick = nt;
    if (base * (n16 / nt) >= enough) break;
  }
  // Small grids (under 3 resident blocks per CU): the busiest CU's share sets the time, so take the
  // tile minimising ceil(blocks / 256) x (NT + 2) (the + 2: a block's fixed patch / epilogue cost in
  // units of one 16-channel n tile). layer4 1x3x3 512 -> 1152 (convbench, 30 clips): NT 8 / 540
  // blocks 0.094 ms, NT 9 / 480 0.082, NT 6 / 720 0.080.
  if (force_nt <= 0 && pick && base * (n16 / pick) < 768) {
    long best = -1;
    for (int nt : {10, 9, 8, 6, 5, 4}) {
      if (n16 % nt) continue;
      const long cost = (base * (n16 / nt) + 255) / 256 * (nt + 2);
      if (best < 0 || cost < best) best = cost, pick = nt;
    }
  }
  return pick;
}

// ---------------------------------------------------------------------------------------------
// conv_patch32_bf16: the spatial 1x3x3 form on v_mfma_f32_32x32x16_bf16 (round 4).
//
// conv_patch_bf16's 16x16x32 tiles read 12 LDS fragments per 20 MFMAs of 16 cycles; a 32x32x16 MFMA
// takes the same cycles per FLOP and each 16-B fragment feeds twice the products, so here a wave
// owns one whole 8x8-pixel output frame (64 voxels = two 32-voxel column blocks) x 32*NB channels:
// per 32-deep K step 2*NB weight + 4 patch fragments for 4*NB MFMAs of 32 cycles (14 per 640 cycles
// at NB = 5 instead of 12 per 320). Block = 4 frames (one per wave) x 8x8 pixels, 256 voxels, so
// each weight byte DMA'd to LDS serves twice the voxels of the 2-frame kernel.
//  * D^T = W . X^T: A operand = 32 weight rows (output channels) x 16 k, B operand = 16 k x 32
//    voxels; lane l (r = l & 31, h = l >> 5) reads row / voxel r, k = 8h .. 8h+7 of the K half;
//  * patch reads are bank-conflict-free: ds_read_b128 serves a wave in the lane groups
//    {0-3,12-15,20-27}, {4-11,16-19,28-31} (and the same +32); lane r of a column block reads
//    voxel vmap(r), which puts each lane group on two whole 8-pixel rows of the frame tile, and the
//    16-B slot q of patch pixel (row, col) is stored at q ^ ((col >> 2 & 1) | (row & 1) << 1):
//    the 4 pixels of a group that share a bank quad (pixel index mod 4, 10-pixel rows) are two
//    columns 4 apart in each of two adjacent rows, so the swizzle separates all four at every tap;
//  * weight rows keep conv_patch_bf16's swizzle (slot q of row n at q ^ g[(n >> 2) & 3]), which is
//    also conflict-free for the 32-row operand's lane groups;
//  * the second 16-deep half of a 32-channel K step is the same address ^ 32 (slot bit 1);
//  * the accumulator of column block cb holds, in register i, channel 32rb + 8(i >> 2) + 4h + (i & 3)
//    of voxel vmap(r): 4 consecutive channels per lane, 8-B bf16 stores as before.
// The weight ring has S = 2 stages (LDS 2 x 25 KiB patch + 2 x NB x 2 KiB: two blocks per CU).

__device__ inline int p32_vmap(int r) {  // lane row r of a 32-voxel column block -> voxel 0..31
  return r < 4 ? r : r < 12 ? r + 12 : r < 16 ? r - 8 : r < 20 ? r + 8 : r < 28 ? r - 12 : r;
}
__device__ inline int p32_swz(int row, int col) { return ((col >> 2) & 1) | ((row & 1) << 1); }

// MODE bit 0: LDS-staged epilogue (the product form); bits 1..5 are convbench knock-outs (timing only):
// 2 no weight DMAs in the loop, 4 no patch DMAs in the loop, 8 no step barriers, 16 no MFMAs,
// 32 no output stores, 64 non-temporal output stores
template <int NB, int S, int OCC, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void conv_patch32_bf16(
    ConvParams p, int n_tiles, int ptw, int npt, int t_tiles) {
  constexpr int FR = 4, TAPS = 9, PC = 10, FPIX = 100;
  constexpr int PIECES = (FR * FPIX + 15) / 16, PBYTES = PIECES * 1024;
  constexpr int WP = 2 * NB;                                   // weight pieces (16 rows x 64 B) per step
  constexpr int PW = (PIECES + 3) / 4, BW = (WP + 3) / 4;      // DMAs per wave (uniform counts)
  constexpr int B_STAGE = WP * 1024, B0 = 2 * PBYTES, SINK = B0 + S * B_STAGE;
  constexpr int LDS = SINK + 1024;
  static_assert(OCC * LDS <= 160 * 1024, "LDS budget");
  static_assert(S >= 2 && S <= TAPS + 1, "wait counts below assume S - 1 <= TAPS");
  __shared__ __align__(16) char smem[LDS];

  const __bf16* x = reinterpret_cast<const __bf16*>(p.x);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  int tile = xcd_swizzle_p(blockIdx.x, gridDim.x);
  const int n0 = (tile % n_tiles) * 32 * NB;
  tile /= n_tiles;
  const int pt = tile % npt;
  tile /= npt;
  const int t0 = (tile % t_tiles) * FR;
  const int clip = tile / t_tiles;
  const int h0 = (pt / ptw) * 8, w0 = (pt % ptw) * 8;
  const int Cin = p.Cin;

  // patch DMA: piece j = wid + 4*i writes pixels 16j .. 16j+15, lane -> pixel 16j + lane/4, physical
  // slot lane & 3 (fetches logical slot (lane & 3) ^ swz); pixels outside the map read the zero block
  int pv[PW];
  unsigned psl[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int pix = (wid + 4 * i) * 16 + (lane >> 2);
    const int f = pix / FPIX, rr = pix - f * FPIX, pr = rr / PC, pc = rr - pr * PC;
    psl[i] = (unsigned)(((lane & 3) ^ p32_swz(pr, pc)) * 16);
    pv[i] = -1;
    if (pix < FR * FPIX) {
      const int ti = t0 + f, hi = h0 - 1 + pr, wi = w0 - 1 + pc;
      if (ti < p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
        pv[i] = ((clip * p.Ti + ti) * p.Hi + hi) * p.Wi + wi;
    }
  }
  auto issue_patch = [&](int c, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wid + 4 * i;
      const void* src = pv[i] >= 0 ? (const void*)(reinterpret_cast<const char*>(x + (size_t)pv[i] * Cin + 32 * c) + psl[i])
                                   : p.zero;
      dma16(src, smem + (j < PIECES ? buf * PBYTES + j * 1024 : SINK));
    }
  };
  const char* wb = reinterpret_cast<const char*>(p.w) + (size_t)n0 * p.Kp * 2;
  unsigned boff[BW];
  {
    const int drow = lane >> 2, dq = (lane & 3) ^ gsw((drow >> 2) & 3);
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      boff[i] = (unsigned)(((j < WP ? j : 0) * 16 + drow) * p.Kp + 8 * dq) * 2u;
    }
  }
  const int nc = Cin / 32;
  auto issue_b = [&](int c, int tap, int slot) __attribute__((always_inline)) {
    const char* base = wb + (size_t)(tap * Cin + 32 * (c < nc ? c : 0)) * 2;
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      dma16(base, boff[i], smem + (j < WP ? B0 + slot * B_STAGE + j * 1024 : SINK));
    }
  };

  f32x16 acc[NB][2];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // patch fragment addresses (K half 0; half 1 is ^ 32) of this lane's voxel in column block cb at
  // every tap, patch buffer 0
  const int vox = p32_vmap(r32);
  int paddr[TAPS][2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int row = 4 * cb + (vox >> 3), col = vox & 7;
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int pr = row + tap / 3, pc = col + tap % 3;
      const int pix = wid * FPIX + pr * PC + pc;
      paddr[tap][cb] = pix * 64 + ((h ^ p32_swz(pr, pc)) << 4);
    }
  }
  const int w_rd0 = B0 + r32 * 64 + ((h ^ gsw((r32 >> 2) & 3)) << 4), w_rd1 = w_rd0 ^ 32;

  issue_patch(0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k) issue_b(k / TAPS, k % TAPS, k);
  int slot = 0;

  for (int c = 0; c < nc; ++c) {
    const bool more = c + 1 < nc;
    const int pbuf = (c & 1) * PBYTES;
    for_taps(std::make_integer_sequence<int, TAPS>{}, [&](auto tc) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tc)::value;
      if constexpr (MODE & 6) {
        vm_wait<0>();
      } else if constexpr (TAP >= 1 && TAP <= S - 1) {
        if (more) vm_wait<(S - 2) * BW + PW>();
        else vm_wait<(S - 2) * BW>();
      } else {
        vm_wait<(S - 2) * BW>();
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(MODE & 8)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      constexpr int T2 = (TAP + S - 1) % TAPS, C2 = (TAP + S - 1) / TAPS;
      const int slot_new = slot == 0 ? S - 1 : slot - 1;
      if constexpr (!(MODE & 2)) issue_b(c + C2, T2, slot_new);
      if constexpr (TAP == 0 && !(MODE & 4)) {
        if (more) issue_patch(c + 1, (c + 1) & 1);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const char* bs = smem + (kk ? w_rd1 : w_rd0) + slot * B_STAGE;
        bf16x8 a[2], b[NB];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          a[cb] = *reinterpret_cast<const bf16x8*>(smem + pbuf + (paddr[TAP][cb] ^ (32 * kk)));
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) b[rb] = *reinterpret_cast<const bf16x8*>(bs + rb * 2048);
#pragma unroll
        for (int rb = 0; rb < NB; ++rb)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            if constexpr (MODE & 16) {
              acc[rb][cb][0] += (float)b[rb][0] * (float)a[cb][kk];
            } else {
              acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[rb], a[cb], acc[rb][cb], 0, 0, 0);
            }
          }
      }
      slot = slot + 1 == S ? 0 : slot + 1;
    });
  }
  vm_wait<0>();

  // epilogue: acc[rb][cb][i] = channel n0 + 32rb + 8(i >> 2) + 4h + (i & 3) of voxel vox of column
  // block cb (frame t0 + wid, frame-tile row 4cb + vox / 8, column vox % 8)
  const __bf16* res = reinterpret_cast<const __bf16*>(p.res);
  __bf16* y = reinterpret_cast<__bf16*>(p.y);
  const int to = t0 + wid;
  // epilogue flags at compile time (MODE 256: residual, 512: ReLU): a runtime flag left both forms of
  // every statement in the code, and their address arithmetic outweighed the main loop's VALU
  constexpr bool RES = (MODE & 256) != 0, RELU = (MODE & 512) != 0;
  auto finish = [&](int rb, int cb, int g, size_t gm) __attribute__((always_inline)) {
    const int n = n0 + 32 * rb + 8 * g + 4 * h;
    f32x4 v = {acc[rb][cb][4 * g], acc[rb][cb][4 * g + 1], acc[rb][cb][4 * g + 2], acc[rb][cb][4 * g + 3]};
    // p.bias is required (patch32_bf16_supported): an unguarded load, so a column block's loads issue
    // together (one vmcnt wait) instead of one guarded load and wait each
    v += gload<f32x4>(p.bias + n);
    if constexpr (RES) {
      const bf16x4 rv = gload<bf16x4>(res + gm * p.Cout + n);
      v += f32x4{(float)rv[0], (float)rv[1], (float)rv[2], (float)rv[3]};
    }
    if constexpr (RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = relu1(v[e]);
    }
    return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  };
  if constexpr (MODE & 32) {  // knock-out: no stores (every accumulator kept live)
    float sum = 0.f;
#pragma unroll
    for (int rb = 0; rb < NB; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) sum += acc[rb][cb][e];
    if (sum == 12345.f) y[lane] = (__bf16)sum;
  } else if constexpr ((MODE & 1) == 0) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int ho = h0 + 4 * cb + (vox >> 3), wo = w0 + (vox & 7);
      if (!(to < p.To && ho < p.Ho && wo < p.Wo)) continue;
      const size_t gm = (((size_t)clip * p.To + to) * p.Ho + ho) * p.Wo + wo;
#pragma unroll
      for (int rb = 0; rb < NB; ++rb)
#pragma unroll
        for (int g = 0; g < 4; ++g) *reinterpret_cast<bf16x4*>(y + gm * p.Cout + n0 + 32 * rb + 8 * g + 4 * h) = finish(rb, cb, g, gm);
    }
  } else {
    // LDS-staged stores: a lane's 8-B pieces are scattered over 32 voxels (32 partial lines per store
    // instruction); staged through the dead patch buffers as [32 voxels][NB*64 B + 16], each column
    // block leaves as NB*2 16-B-per-lane stores of whole voxel segments (contiguous 8-pixel rows
    // when the block covers every channel). Store addresses: a wave-uniform base (clip, frame, first
    // row of the column block) plus a small per-lane offset.
    constexpr int SEG = NB * 64, VS = SEG + 16, INS = SEG * 32 / 1024;
    static_assert(4 * 32 * VS <= 2 * PBYTES, "staging fits the patch buffers");
    char* st = smem + wid * 32 * VS;
    const bool full = to < p.To && h0 + 8 <= p.Ho && w0 + 8 <= p.Wo;  // wave-uniform
    const int row_el = p.Wo * p.Cout;                                 // elements per map row
    __builtin_amdgcn_s_barrier();  // every wave is past its last patch / weight read
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int ho_l = h0 + 4 * cb + (vox >> 3), wo_l = w0 + (vox & 7);
      size_t gm_l = 0;
      if constexpr (RES)
        gm_l = (((size_t)clip * p.To + (to < p.To ? to : 0)) * p.Ho + (ho_l < p.Ho ? ho_l : 0)) * p.Wo +
               (wo_l < p.Wo ? wo_l : 0);
#pragma unroll
      for (int rb = 0; rb < NB; ++rb)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(st + vox * VS + (32 * rb + 8 * g + 4 * h) * 2) = finish(rb, cb, g, gm_l);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      __bf16* yb = y + ((((size_t)clip * p.To + to) * p.Ho + h0 + 4 * cb) * p.Wo + w0) * p.Cout + n0;
#pragma unroll
      for (int k = 0; k < INS; ++k) {
        const int e = 1024 * k + 16 * lane, v = e / SEG, off = e - v * SEG;
        const bf16x8 val = *reinterpret_cast<const bf16x8*>(st + v * VS + off);
        const int r = v >> 3, c = v & 7;
        __bf16* dst = yb + (r * row_el + c * p.Cout + off / 2);
        if (full || (to < p.To && h0 + 4 * cb + r < p.Ho && w0 + c < p.Wo)) {
          if constexpr (MODE & 64) {
            __builtin_nontemporal_store(val, reinterpret_cast<bf16x8*>(dst));
          } else {
            *reinterpret_cast<bf16x8*>(dst) = val;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
  }
}

template <int NB, int S = 2>
constexpr int patch32_occ() {
  constexpr int lds = 2 * 25 * 1024 + S * NB * 2048 + 1024;
  constexpr int occ = 160 * 1024 / lds;
  return occ > 4 ? 4 : occ;
}

template <int NB, int S, int MODE>
hipError_t launch_p32_m(const ConvParams& p, hipStream_t s) {
  const PatchGrid g = patch_grid(p, 4);
  const int n_tiles = p.Cout / (32 * NB);
  hipLaunchKernelGGL((conv_patch32_bf16<NB, S, patch32_occ<NB, S>(), MODE>), dim3((unsigned)(g.base * n_tiles)), dim3(256),
                     0, s, p, n_tiles, g.ptw, g.npt, g.tt);
  return hipGetLastError();
}

// EPI: MODE bits 0..6 (1 = the staged product epilogue); the residual / ReLU bits come from p
template <int NB, int S = 2, int EPI = 1>
hipError_t launch_p32(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 0: return launch_p32_m<NB, S, EPI>(p, s);
    case 1: return launch_p32_m<NB, S, EPI | 256>(p, s);
    case 2: return launch_p32_m<NB, S, EPI | 512>(p, s);
    default: return launch_p32_m<NB, S, EPI | 768>(p, s);
  }
}

// N tile (32-channel blocks). Product rule, per clip: the widest of NB = 5, 4, 3 (160-, 128-, 96-channel
// blocks) that divides Cout / 32 and gives ONE CLIP >= 24 blocks -- layer1's 64 -> 160 (NB 5: 392 blocks
// per 32x112x112 clip), layer2's 128 -> 256 (NB 4) and 128 -> 288 (NB 3), layer3's 256 -> 480 (NB 5) and
// 256 -> 576 (NB 3); layer4's 7x7 maps give 9-12 and stay on conv_patch_bf16. Round 6 (convbench, 30
// clips, profiles/r06k_patch32_layer234.txt): layer2 0.241 vs conv_patch_bf16's 0.268 ms (256) and 0.303
// vs 0.307 (288), layer3 0.115 vs 0.126 (480) and 0.146 vs 0.155 (576), layer4 0.086 vs 0.082 (round 4
// had found conv_patch_bf16 as fast or faster on layer2-4, before both kernels' store and DMA work);
// bit-identical. 0: not taken. force_nb > 0 (convbench, CLASFV_PATCH_NT = -NB) takes any NB that divides.
// The rule counts blocks per clip, never the batch's, so whether a clip's convs run 32x32x16 or
// 16x16x32 products does not depend on how many clips share the launch (the two are bit-identical
// anyway). On small batches it costs nothing: with the round-5 kernels conv_patch32_bf16 is the faster
// form at every batch size (layer1, with the residual: N = 1 0.032 vs 0.044 ms, N = 4 0.105 vs 0.151,
// N = 30 0.756 vs 1.013; profiles/r06j_patch32_small_batch.txt).
int patch32_pick_nb(const ConvParams& p, int force_nb) {
  if (p.Cout % 32) return 0;
  const int n32 = p.Cout / 32;
  if (force_nb > 0) return (force_nb <= 5 && force_nb >= 2 && n32 % force_nb == 0) ? force_nb : 0;
  const long per_clip = patch_grid(p, 4).base / p.N;  // frame blocks x 8x8 tiles of one clip
  for (int nb : {5, 4, 3})
    if (n32 % nb == 0 && per_clip * (n32 / nb) >= 24) return nb;
  return 0;
}

}  // namespace

bool patch32_bf16_supported(const ConvParams& p) {
  if (!p.in_bf16 || !p.out_bf16 || p.stem || p.x2 || !p.bias) return false;
  if (p.st != 1 || p.sh != 1 || p.sw != 1) return false;
  if (!(p.KT == 1 && p.KH == 3 && p.KW == 3 && p.pt == 0 && p.ph == 1 && p.pw == 1)) return false;
  if (p.Cin % 32 || p.Kp != 9 * p.Cin) return false;
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi) return false;
  if (patch32_pick_nb(p, p.patch_nt < 0 ? -p.patch_nt : 0) == 0) return false;
  if ((long)p.N * p.Ti * p.Hi * p.Wi >= (1L << 31) / 2) return false;
  return true;
}

hipError_t launch_patch32_bf16(const ConvParams& p, hipStream_t s) {
  if (!patch32_bf16_supported(p)) return hipErrorInvalidValue;
  const int nb = patch32_pick_nb(p, p.patch_nt < 0 ? -p.patch_nt : 0);  // CLASFV_PATCH_NT < 0: force NB
  // output stores non-temporal (MODE 64): the forward's bf16 A/B (profiles/r05ad_nt_stores_ab3.txt)
  // 3151 / 3166 -> 3201 / 3203 clips/s, this kernel 2.03 -> 1.98 ms and its consumer conv_patch_bf16
  // faster too; CLASFV_PATCH32_CACHED_STORES keeps the cached form
  if (!(p.vflags & CLASFV_VARIANT_PATCH32_CACHED_STORES) && nb == 5) return launch_p32<5, 2, 1 | 64>(p, s);
  switch (nb) {
    case 5: return launch_p32<5>(p, s);
    case 4: return launch_p32<4>(p, s);
    case 3: return launch_p32<3>(p, s);
    case 2: return launch_p32<2>(p, s);
  }
  return hipErrorInvalidValue;
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: epi = MODE (0 = direct 8-B stores from the accumulator layout, 1 = LDS-staged,
// odd values above 1: knock-outs at NB 5)
hipError_t launch_patch32_bf16_epi(const ConvParams& p, hipStream_t s, int epi) {
  if (!patch32_bf16_supported(p)) return hipErrorInvalidValue;
  const int nb = patch32_pick_nb(p, p.patch_nt < 0 ? -p.patch_nt : 0);
  if (epi == 1) return launch_patch32_bf16(p, s);
  if (epi == 0) {
    switch (nb) {
      case 5: return launch_p32<5, 2, 0>(p, s);
      case 4: return launch_p32<4, 2, 0>(p, s);
      case 3: return launch_p32<3, 2, 0>(p, s);
      case 2: return launch_p32<2, 2, 0>(p, s);
    }
  }
  if (nb != 5) return hipErrorInvalidValue;
  switch (epi) {  // knock-outs (MODE bits), NB 5
    case 3: return launch_p32<5, 2, 3>(p, s);
    case 5: return launch_p32<5, 2, 5>(p, s);
    case 7: return launch_p32<5, 2, 7>(p, s);
    case 9: return launch_p32<5, 2, 9>(p, s);
    case 15: return launch_p32<5, 2, 15>(p, s);
    case 17: return launch_p32<5, 2, 17>(p, s);
    case 33: return launch_p32<5, 2, 33>(p, s);
    case 47: return launch_p32<5, 2, 47>(p, s);
    case 31: return launch_p32<5, 2, 31>(p, s);
    case 65: return launch_p32<5, 2, 65>(p, s);
  }
  return hipErrorInvalidValue;
}
#endif

// ---------------------------------------------------------------------------------------------
// (convbench only, round 6: measured no faster than conv_dma_w -- layer2 0.390-0.396 vs 0.399 ms,
// layer3 0.143-0.145 vs 0.145, layer4 0.075-0.081 vs 0.067; profiles/r06b_patch_s2_bf16.txt)
#ifdef CLASFV_KNOCKOUTS
// conv_patch_s2_bf16 (round 6): the strided spatial convs (1x3x3, stride (1,2,2), pad (0,1,1)) of the
// Conv2Plus1D first halves of layer2-4 (torchvision Conv2Plus1D via src/model/R2plus1D_18_MotionNet.py:33-37)
// in the bf16 engines. conv_dma_w gathers one 128-B tap row per output voxel and tap (9 x 64 rows per
// 8x8 output tile and 32 channels); here a block DMAs the tile's 17x17-pixel input patch once per
// 32-channel chunk (289 rows) and every tap reads its A fragments from it.
//  * polyphase patch: the patch is stored as its 4 (row, column) parity sub-grids of 9 x 9 slots
//    (phase-1 grids use 8 x 8 of them). Tap (kh, kw) of output pixel (oy, ox) reads input (2 oy + kh,
//    2 ox + kw) = sub-grid (kh & 1, kw & 1), slot (oy + kh / 2, ox + kw / 2): every tap reads runs of
//    consecutive slots, as a stride-1 conv does, and the 16-B slot q of slot (row sr, col sc) is stored
//    at q ^ 2 (sr & 1) -- conflict-free for every tap's ds_read_b128 lane groups (the two output rows
//    of a 16-voxel m tile sit on sub-grid rows of opposite parity);
//  * sub-grid-major LDS image [4 sub-grids][FR frames][81 slots] (each sub-grid image padded to whole
//    1-KiB DMA pieces), ONE buffer: the taps run sub-grid by sub-grid -- (0,0) (0,2) (2,0) (2,2), then
//    (0,1) (2,1), (1,0) (1,2), (1,1) -- and each sub-grid of the next chunk is DMA'd as soon as the
//    step barrier shows every wave past its last tap (5-8 steps before it is read), so the patch is
//    single-buffered and two blocks fit a CU;
//  * the rest is conv_patch_bf16: 16x16x32 MFMAs with D^T = W . A^T, wave w owns m tiles MT w ..
//    MT w + MT - 1 (FR frames x 64 voxels per block), B ring of S stages (weights w[n][tap Cin + c],
//    conv_dma's image), LDS-staged epilogue.
// K order: chunk-major, then the tap order above: not conv_dma_w's (tap-major) fp32 summation order,
// so outputs match it within bf16 rounding, not bit for bit.
namespace {

constexpr int S2_ORDER[9] = {0, 2, 6, 8, 1, 7, 3, 5, 4};  // tap (kh * 3 + kw) of each step of a chunk

template <int FR>
struct S2Geo {
  static constexpr int PITCH = 9, SUB = 81;                    // sub-grid slots: 9 rows x 9 columns
  static constexpr int SUBP = (FR * SUB + 15) / 16;            // 1-KiB pieces per sub-grid image
  static constexpr int PW = (SUBP + 3) / 4;                    // DMAs per wave per sub-grid image
  static constexpr int SUBB = SUBP * 1024;                     // bytes per sub-grid image
  static constexpr int BYTES = 4 * SUBB;
};

template <int NT, int FR, int S, int OCC, int EF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void conv_patch_s2_bf16(
    ConvParams p, int n_tiles, int ptw, int npt, int t_tiles) {
  using G = S2Geo<FR>;
  constexpr int MT = FR, PW = G::PW, BW = (NT + 3) / 4;
  constexpr int B_STAGE = NT * 1024, B0 = G::BYTES, SINK = B0 + S * B_STAGE;
  constexpr int LDS = SINK + 1024;
  static_assert(OCC * LDS <= 160 * 1024, "LDS budget");
  static_assert(S == 2 || S == 3, "wait counts below");
  __shared__ __align__(16) char smem[LDS];

  const __bf16* x = reinterpret_cast<const __bf16*>(p.x);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, l16 = lane & 15;
  int tile = xcd_swizzle_p(blockIdx.x, gridDim.x);
  const int n0 = (tile % n_tiles) * 16 * NT;
  tile /= n_tiles;
  const int pt = tile % npt;
  tile /= npt;
  const int t0 = (tile % t_tiles) * FR;
  const int clip = tile / t_tiles;
  const int h0 = (pt / ptw) * 8, w0 = (pt % ptw) * 8;  // output tile origin
  const int Cin = p.Cin;

  // patch DMA of one sub-grid image: piece j = wid + 4 i writes slots 16 j .. 16 j + 15 of it, lane ->
  // slot 16 j + lane / 4 = frame f, row sr, column sc; pieces past the image land in the sink, slots
  // past the patch (the phase-1 grids' ninth row / column) read the zero block
  int pv[4][PW];
  unsigned psl[4][PW];
#pragma unroll
  for (int sg = 0; sg < 4; ++sg)
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int slot = (wid + 4 * i) * 16 + (lane >> 2);
      const int f = slot / G::SUB, r = slot - f * G::SUB, sr = r / G::PITCH, sc = r - sr * G::PITCH;
      const int pr = 2 * sr + (sg >> 1), pc = 2 * sc + (sg & 1);
      psl[sg][i] = (unsigned)(((lane & 3) ^ (2 * (sr & 1))) * 16);
      pv[sg][i] = -1;
      const int ti = t0 + f, hi = 2 * h0 - 1 + pr, wi = 2 * w0 - 1 + pc;
      if (f < FR && pr <= 16 && pc <= 16 && ti < p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
        pv[sg][i] = ((clip * p.Ti + ti) * p.Hi + hi) * p.Wi + wi;
    }
  auto issue_sub = [&](int c, int sg) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wid + 4 * i;
      const void* src = pv[sg][i] >= 0
                            ? (const void*)(reinterpret_cast<const char*>(x + (size_t)pv[sg][i] * Cin + 32 * c) + psl[sg][i])
                            : p.zero;
      dma16(src, smem + (j < G::SUBP ? sg * G::SUBB + j * 1024 : SINK));
    }
  };
  const char* wb = reinterpret_cast<const char*>(p.w) + (size_t)n0 * p.Kp * 2;
  unsigned boff[BW];
  {
    const int drow = lane >> 2, dq = (lane & 3) ^ gsw((drow >> 2) & 3);
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      boff[i] = (unsigned)(((j < NT ? j : 0) * 16 + drow) * p.Kp + 8 * dq) * 2u;
    }
  }
  const int nc = Cin / 32;
  auto issue_b = [&](int c, int tap, int slot) __attribute__((always_inline)) {
    const char* base = wb + (size_t)(tap * Cin + 32 * (c < nc ? c : 0)) * 2;
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const int j = wid + 4 * i;
      dma16(base, boff[i], smem + (j < NT ? B0 + slot * B_STAGE + j * 1024 : SINK));
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragment i of this lane: block voxel m = 16 (MT wid + i) + l16 = frame f, pixel (oy, ox) of the
  // 8x8 tile; LDS byte address of its 16-B slot q at every tap
  int aaddr[9][MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = 16 * (MT * wid + i) + l16, f = m >> 6, px = m & 63, oy = px >> 3, ox = px & 7;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3, sg = ((kh & 1) << 1) | (kw & 1);
      const int sr = oy + (kh >> 1), sc = ox + (kw >> 1);
      const int slot = f * G::SUB + sr * G::PITCH + sc;
      aaddr[tap][i] = sg * G::SUBB + slot * 64 + ((q ^ (2 * (sr & 1))) << 4);
    }
  }
  const int b_rd = B0 + l16 * 64 + (q ^ gsw(l16 >> 2)) * 16;

  // prologue: sub-grids (0,0), (0,1), (1,0) of chunk 0 (sub-grid (1,1) goes out at chunk 0's step 0),
  // then the first S - 1 weight steps
  issue_sub(0, 0);
  issue_sub(0, 1);
  issue_sub(0, 2);
#pragma unroll
  for (int k = 0; k < S - 1; ++k) issue_b(k / 9, S2_ORDER[k % 9], k);
  int slot = 0;

  for (int c = 0; c < nc; ++c) {
    const bool more = c + 1 < nc;
    for_taps(std::make_integer_sequence<int, 9>{}, [&](auto tc) __attribute__((always_inline)) {
      constexpr int T = decltype(tc)::value;
      // Each step issues B(step + S - 1), then at most one sub-grid image: step 0 sub-grid (1,1) of
      // this chunk, steps 4 / 6 / 8 sub-grids (0,0) / (0,1) / (1,0) of the next. A step needs B(step)
      // and, at steps 0 / 4 / 6 / 8, a sub-grid image issued 5-8 steps earlier -- older than B(step)
      // -- so it may leave in flight what was issued after B(step): the images of the last S - 1
      // steps and (S = 3) one weight step.
      constexpr int TP1 = (T + 8) % 9, TP2 = (T + 7) % 9;  // the previous two steps' tap positions
      auto img = [&](int tp, bool same_chunk_more, bool prev_chunk) -> int {
        // sub-grid DMAs issued at step position tp (of this chunk if !prev_chunk, else of the last)
        if (tp == 0) return PW;
        if (tp == 4 || tp == 6 || tp == 8) return (prev_chunk ? true : same_chunk_more) ? PW : 0;
        return 0;
      };
      if constexpr (S == 2) {
        const int n = T == 0 ? (c > 0 ? img(TP1, more, true) : 0) : img(TP1, more, false);
        if (n) vm_wait<PW>(); else vm_wait<0>();
      } else {
        const int n1 = T == 0 ? (c > 0 ? img(TP1, more, true) : 0) : img(TP1, more, false);
        const int n2 = T <= 1 ? (c > 0 ? img(TP2, more, true) : 0) : img(TP2, more, false);
        const int n = n1 + n2;
        if (n == 2 * PW) vm_wait<BW + 2 * PW>();
        else if (n == PW) vm_wait<BW + PW>();
        else vm_wait<BW>();
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      constexpr int T2 = (T + S - 1) % 9, C2 = (T + S - 1) / 9;
      const int slot_new = slot == 0 ? S - 1 : slot - 1;  // (s + S - 1) % S
      issue_b(c + C2, S2_ORDER[T2], slot_new);
      if constexpr (T == 0) issue_sub(c, 3);
      if constexpr (T == 4) { if (more) issue_sub(c + 1, 0); }
      if constexpr (T == 6) { if (more) issue_sub(c + 1, 1); }
      if constexpr (T == 8) { if (more) issue_sub(c + 1, 2); }
      constexpr int TAP = S2_ORDER[T];
      bf16x8 a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = *reinterpret_cast<const bf16x8*>(smem + aaddr[TAP][i]);
      const char* bs = smem + b_rd + slot * B_STAGE;
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + j * 1024);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      slot = slot + 1 == S ? 0 : slot + 1;
    });
  }
  vm_wait<0>();  // the past-the-end B fetches land before the block's LDS is released

  // epilogue (conv_patch_bf16's LDS-staged stores): acc[i][j] = channels n0 + 16 j + 4 q .. + 3 of
  // block voxel 16 (MT wid + i) + l16
  const __bf16* res = reinterpret_cast<const __bf16*>(p.res);
  __bf16* y = reinterpret_cast<__bf16*>(p.y);
  auto finish = [&](int i, int j, size_t gm) __attribute__((always_inline)) {
    const int n = n0 + j * 16 + 4 * q;
    f32x4 v = acc[i][j] + gload<f32x4>(p.bias + n);
    if constexpr (EF & 1) {
      const bf16x4 r = gload<bf16x4>(res + gm * p.Cout + n);
      v += f32x4{(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
    }
    if constexpr (EF & 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = relu1(v[e]);
    }
    return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  };
  constexpr int SEG = NT * 32, VS = SEG + 16;
  constexpr int MH = 4 * 16 * MT * VS <= LDS ? MT : 1, INS = 16 * MH * SEG / 1024;
  static_assert(4 * 16 * MH * VS <= LDS, "staging fits the block's LDS");
  static_assert(16 * MH * SEG % 1024 == 0, "whole store instructions");
  char* st = smem + wid * 16 * MH * VS;
  __builtin_amdgcn_s_barrier();  // every wave is past its last patch / weight read
#pragma unroll
  for (int i0 = 0; i0 < MT; i0 += MH) {
#pragma unroll
    for (int i = i0; i < i0 + MH; ++i) {
      size_t gm = 0;
      if constexpr (EF & 1) {
        const int m = 16 * (MT * wid + i) + l16, f = m >> 6, px = m & 63, to = t0 + f;
        const int ho = h0 + (px >> 3), wo = w0 + (px & 7);
        gm = (((size_t)clip * p.To + (to < p.To ? to : 0)) * p.Ho + (ho < p.Ho ? ho : 0)) * p.Wo + (wo < p.Wo ? wo : 0);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
        *reinterpret_cast<bf16x4*>(st + (16 * (i - i0) + l16) * VS + (16 * j + 4 * q) * 2) = finish(i, j, gm);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const int mp = 16 * (MT * wid + i0), f = mp >> 6, px0 = mp & 63, to = t0 + f;
    __bf16* yb = y + ((((size_t)clip * p.To + to) * p.Ho + h0 + px0 / 8) * p.Wo + w0) * p.Cout + n0;
    const bool full = to < p.To && h0 + px0 / 8 + 2 * MH <= p.Ho && w0 + 8 <= p.Wo;
    const int row_el = p.Wo * p.Cout;
#pragma unroll
    for (int k = 0; k < INS; ++k) {
      const int e = 1024 * k + 16 * lane, v = e / SEG, off = e - v * SEG;
      const bf16x8 val = *reinterpret_cast<const bf16x8*>(st + v * VS + off);
      const int lo = (v >> 3) * row_el + (v & 7) * p.Cout + off / 2;
      if (full || (to < p.To && h0 + px0 / 8 + (v >> 3) < p.Ho && w0 + (v & 7) < p.Wo))
        *reinterpret_cast<bf16x8*>(yb + lo) = val;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  }
}

template <int NT, int FR, int S>
constexpr int s2_occ() {
  constexpr int lds = S2Geo<FR>::BYTES + S * NT * 1024 + 1024;
  constexpr int occ = 160 * 1024 / lds;
  return occ > 4 ? 4 : occ;
}

struct S2Grid {
  int ptw, npt, tt;
  long base;  // blocks per n tile
};

S2Grid s2_grid(const ConvParams& p, int fr) {
  S2Grid g{};
  g.ptw = (p.Wo + 7) / 8;
  g.npt = g.ptw * ((p.Ho + 7) / 8);
  g.tt = (p.To + fr - 1) / fr;
  g.base = (long)p.N * g.tt * g.npt;
  return g;
}

template <int NT, int FR, int S, int EF>
hipError_t launch_s2_e(const ConvParams& p, hipStream_t s) {
  const S2Grid g = s2_grid(p, FR);
  const int n_tiles = p.Cout / (16 * NT);
  hipLaunchKernelGGL((conv_patch_s2_bf16<NT, FR, S, s2_occ<NT, FR, S>(), EF>), dim3((unsigned)(g.base * n_tiles)),
                     dim3(256), 0, s, p, n_tiles, g.ptw, g.npt, g.tt);
  return hipGetLastError();
}

template <int NT, int FR = 2, int S = 2>
hipError_t launch_s2(const ConvParams& p, hipStream_t s) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 0: return launch_s2_e<NT, FR, S, 0>(p, s);
    case 1: return launch_s2_e<NT, FR, S, 1>(p, s);
    case 2: return launch_s2_e<NT, FR, S, 2>(p, s);
    default: return launch_s2_e<NT, FR, S, 3>(p, s);
  }
}

// N tile: the widest dividing Cout/16 with about two blocks per CU (>= 512 blocks); small grids take the
// tile minimising ceil(blocks / 512) x (NT + 2) (two resident blocks per CU), as patch_pick_nt.
// Per-clip shape rule: the choice depends on the batch only through the block count, and every NT runs
// the same per-voxel products in the same order (bit-identical across NT).
int s2_pick_nt(const ConvParams& p, int force_nt) {
  const int n16 = p.Cout / 16;
  const long base = s2_grid(p, 2).base;
  int pick = 0;
  for (int nt : {10, 8, 6, 5, 4}) {
    if (n16 % nt) continue;
    if (force_nt > 0) {
      if (nt == force_nt) return nt;
      continue;
    }
    if (!pick) pick = nt;
    if (base * (n16 / nt) >= 512) return nt;
  }
  if (!pick || force_nt > 0) return 0;
  long best = -1;
  for (int nt : {10, 8, 6, 5, 4}) {
    if (n16 % nt) continue;
    const long cost = (base * (n16 / nt) + 511) / 512 * (nt + 2);
    if (best < 0 || cost < best) best = cost, pick = nt;
  }
  return pick;
}

}  // namespace

bool patch_s2_bf16_supported(const ConvParams& p) {
  if (!p.in_bf16 || !p.out_bf16 || p.stem || p.x2 || !p.bias) return false;
  if (!(p.KT == 1 && p.KH == 3 && p.KW == 3 && p.st == 1 && p.sh == 2 && p.sw == 2 && p.pt == 0 && p.ph == 1 && p.pw == 1))
    return false;
  if (p.Cin % 32 || p.Cout % 16 || p.Kp != 9 * p.Cin) return false;
  if (p.To != p.Ti || p.Ho != (p.Hi + 1) / 2 || p.Wo != (p.Wi + 1) / 2) return false;
  if (s2_pick_nt(p, p.patch_nt) == 0) return false;
  if ((long)p.N * p.Ti * p.Hi * p.Wi >= (1L << 31) / 2) return false;
  return true;
}

hipError_t launch_patch_s2_bf16(const ConvParams& p, hipStream_t s) {
  if (!patch_s2_bf16_supported(p)) return hipErrorInvalidValue;
  switch (s2_pick_nt(p, p.patch_nt)) {
    case 10: return launch_s2<10>(p, s);
    case 8: return launch_s2<8>(p, s);
    case 6: return launch_s2<6>(p, s);
    case 5: return launch_s2<5>(p, s);
    case 4: return launch_s2<4>(p, s);
  }
  return hipErrorInvalidValue;
}

// tools/convbench: ko = S * 100 + FR * 10 (+ NT forced through CLASFV_PATCH_NT / CB patch_nt)
hipError_t launch_patch_s2_bf16_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (!patch_s2_bf16_supported(p)) return hipErrorInvalidValue;
  const int nt = s2_pick_nt(p, p.patch_nt), st = ko / 100, fr = ko / 10 % 10;
  auto go = [&](auto ntc) -> hipError_t {
    constexpr int NT = decltype(ntc)::value;
    if (st == 3 && fr == 2) return launch_s2<NT, 2, 3>(p, s);
    if constexpr (NT % 2 == 0) {  // FR 1: one m tile per wave (whole staged store instructions need even NT)
      if (st == 2 && fr == 1) return launch_s2<NT, 1, 2>(p, s);
      if (st == 3 && fr == 1) return launch_s2<NT, 1, 3>(p, s);
    }
    if (fr == 1) return hipErrorInvalidValue;
    return launch_s2<NT, 2, 2>(p, s);
  };
  switch (nt) {
    case 10: return go(std::integral_constant<int, 10>{});
    case 8: return go(std::integral_constant<int, 8>{});
    case 6: return go(std::integral_constant<int, 6>{});
    case 5: return go(std::integral_constant<int, 5>{});
    case 4: return go(std::integral_constant<int, 4>{});
  }
  return hipErrorInvalidValue;
}
#endif  // CLASFV_KNOCKOUTS

bool patch_bf16_supported(const ConvParams& p) {
  if (!p.in_bf16 || !p.out_bf16 || p.stem || p.x2) return false;
  if (p.st != 1 || p.sh != 1 || p.sw != 1) return false;
  const bool spatial = p.KT == 1 && p.KH == 3 && p.KW == 3 && p.pt == 0 && p.ph == 1 && p.pw == 1;
  const bool temporal = p.KT == 3 && p.KH == 1 && p.KW == 1 && p.pt == 1 && p.ph == 0 && p.pw == 0;
  if (!spatial && !temporal) return false;
  if (p.Cin % 32 || p.Cout % 16 || p.Kp != p.KT * p.KH * p.KW * p.Cin) return false;
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi) return false;
  if (patch_pick_nt(p, 0) == 0) return false;
  // voxel indices are int32 in the kernel
  if ((long)p.N * p.Ti * p.Hi * p.Wi >= (1L << 31) / 2) return false;
  return true;
}

hipError_t launch_patch_bf16(const ConvParams& p, hipStream_t s) {
  if (!patch_bf16_supported(p)) return hipErrorInvalidValue;
  const int nt = patch_pick_nt(p, p.patch_nt);
  return p.KT == 1 ? launch_nt<1>(p, nt, s) : launch_nt<3>(p, nt, s);
}


#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip variant sweep: ko = FR*1000 + S*100 + NT (e.g. 2305 = 2 frames per block,
// 3 ring stages, NT 5)
namespace {
template <int KT, int FR, int S>
hipError_t ko_nt(const ConvParams& p, int nt, hipStream_t s) {
  switch (nt) {
    case 10: if constexpr (patch_occ<10, KT, FR, S>() >= 1) return launch_p<10, KT, FR, S>(p, s); break;
    case 9: if constexpr (patch_occ<9, KT, FR, S>() >= 1) return launch_p<9, KT, FR, S>(p, s); break;
    case 8: if constexpr (patch_occ<8, KT, FR, S>() >= 1) return launch_p<8, KT, FR, S>(p, s); break;
    case 6: return launch_p<6, KT, FR, S>(p, s);
    case 5: return launch_p<5, KT, FR, S>(p, s);
    case 4: return launch_p<4, KT, FR, S>(p, s);
  }
  return hipErrorInvalidValue;
}
template <int KT, int FR>
hipError_t ko_s(const ConvParams& p, int st, int nt, hipStream_t s) {
  switch (st) {
    case 2: return ko_nt<KT, FR, 2>(p, nt, s);
    case 3: return ko_nt<KT, FR, 3>(p, nt, s);
    case 4: return ko_nt<KT, FR, 4>(p, nt, s);
  }
  if constexpr (KT == 1) {
    if (st == 5) return ko_nt<KT, FR, 5>(p, nt, s);
    if (st == 6) return ko_nt<KT, FR, 6>(p, nt, s);
  }
  return hipErrorInvalidValue;
}
// the product configuration with the direct (unstaged) epilogue
template <int KT>
hipError_t direct_nt(const ConvParams& p, int nt, hipStream_t s) {
  constexpr int FR = product_fr<KT>(), S = product_s<KT>();
  switch (nt) {
    case 10: return launch_p<10, KT, FR, S, false>(p, s);
    case 9: return launch_p<9, KT, FR, S, false>(p, s);
    case 8: return launch_p<8, KT, FR, S, false>(p, s);
    case 6: return launch_p<6, KT, FR, S, false>(p, s);
    case 5: return launch_p<5, KT, FR, S, false>(p, s);
    case 4: return launch_p<4, KT, FR, S, false>(p, s);
  }
  return hipErrorInvalidValue;
}
}  // namespace

// ko 10000: the product configuration with direct 8-B output stores (no LDS staging)
hipError_t launch_patch_bf16_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (ko == 0) return launch_patch_bf16(p, s);
  if (ko == 10000) {
    if (!patch_bf16_supported(p)) return hipErrorInvalidValue;
    const int nt = patch_pick_nt(p, p.patch_nt);
    return p.KT == 1 ? direct_nt<1>(p, nt, s) : direct_nt<3>(p, nt, s);
  }
  const int fr = ko / 1000, st = ko / 100 % 10, nt = ko % 100;
  if (p.Cout % (16 * nt)) return hipErrorInvalidValue;
  if (fr == 2) return p.KT == 1 ? ko_s<1, 2>(p, st, nt, s) : ko_s<3, 2>(p, st, nt, s);
  if (fr == 4) return p.KT == 1 ? ko_s<1, 4>(p, st, nt, s) : ko_s<3, 4>(p, st, nt, s);
  return hipErrorInvalidValue;
}
#endif
