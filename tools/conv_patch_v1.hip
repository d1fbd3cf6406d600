// Round-2 copy of the previous conv_patch kernel (2 frames x 8x8 tile, 2 m tiles per wave), kept
// only as the convbench A/B baseline (tools/convbench.hip kind spp, ko 901).
// Patch-staged bf16 implicit GEMM for the stride-1 1x3x3 spatial convs of the R(2+1)D-18 encoder
// (torchvision Conv2Plus1D spatial half, called from src/model/R2plus1D_18_MotionNet.py:29-37),
// BASELINE config[4] (bf16 activations/weights, fp32 accumulation).
//
// Why: conv_dma (conv.hip) gathers the im2col A tile straight from global memory, so every input
// voxel crosses the L2 -> LDS path once per 3x3 tap; in bf16 the MFMAs are 16x faster than in fp32
// and that gather, not the matrix cores, sets the time (layer1 64->160: 2.08 ms, 267 TF alg.).
// Here a block's output tile is 2 frames x 8 rows x 8 columns (128 voxels); for each 32-channel
// chunk the 2 x 10 x 10 input patch (200 voxels x 64 B) is copied to LDS ONCE and the nine taps
// read their A fragments from it at pixel offsets kh*10 + kw: 9 x 128 gathered rows become 200.
//  * K order: chunk-major, tap-minor (step s = 9*chunk + tap); weights keep conv_dma's image
//    [Cout_alloc][Kp] with k = tap*Cin + c, so one B row segment is w[n][tap*Cin + 32*chunk ..];
//  * patch image: double-buffered, pixel rows of 64 B, 16-B slot q of pixel p stored at
//    q ^ g[(p >> 2) & 3] (the tap shift makes some reads 2-way conflicted; B reads are conflict-free);
//  * B ring: 3 stages of NT x 16 rows x 64 B, one per step, as in conv_dma; all copies are
//    LDS-DMA (global_load_lds_dwordx4) with per-lane source addresses (zero block for halo pixels);
//  * counted vmcnt: at step s a wave waits for its own B(s) (and, implied by in-order completion,
//    the patch of the step's chunk), then a block barrier; the next chunk's patch is issued at the
//    chunk's tap 0, after the barrier that retires the buffer's previous chunk;
//  * epilogue: the MFMAs compute D^T = W . A^T, so a lane holds 4 consecutive output channels of
//    one voxel: folded-BN bias, optional residual, ReLU, 8-B bf16 stores; voxels outside the map
//    (ragged 28/14/7-pixel maps) are masked.
#include <hip/hip_bf16.h>
#include <stdlib.h>

#include "../fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd/csrc/common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int PT = 2, PR = 8, PC = 8;             // output tile (frames, rows, columns)
constexpr int QR = PR + 2, QC = PC + 2;           // input patch rows / columns (3x3 halo)
constexpr int PPIX = PT * QR * QC;                // 200 patch pixels
constexpr int P_INS = (PPIX * 64 + 1023) / 1024;  // 13 DMA pieces of 1 KiB
constexpr int P_PW = (P_INS + 3) / 4;             // 4 pieces per wave (tail pieces fill the pad)
constexpr int P_BYTES = 4 * P_PW * 1024;          // 16 KiB per patch buffer

// slot swizzle g = {0, 2, 3, 1} as arithmetic: a runtime-indexed constant array is a global load,
// and its in-order vmcnt wait would drain the whole DMA ring in front of every A read
__device__ inline int gsw(int i) { return (0x78 >> (2 * i)) & 3; }

__device__ inline int xcd_swizzle_p(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

template <int NT>
__global__ __launch_bounds__(256) void conv_patch_bf16(ConvParams p, int n_tiles, int tiles_w, int tiles_h, int tiles_t) {
  constexpr int BN = 16 * NT, S = 3;
  constexpr int B_PW = (NT + 3) / 4;
  constexpr int B_STAGE = NT * 1024;
  constexpr int B0 = 2 * P_BYTES;
  constexpr int JUNK = B0 + S * B_STAGE;
  __shared__ __align__(16) char smem[JUNK + 1024];

  const __bf16* x = reinterpret_cast<const __bf16*>(p.x);
  const __bf16* w = reinterpret_cast<const __bf16*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tile = xcd_swizzle_p(blockIdx.x, gridDim.x);
  const int n0 = (tile % n_tiles) * BN;
  tile /= n_tiles;
  const int w0 = (tile % tiles_w) * PC;
  tile /= tiles_w;
  const int h0 = (tile % tiles_h) * PR;
  tile /= tiles_h;
  const int t0 = (tile % tiles_t) * PT;
  const int nclip = tile / tiles_t;
  const int q = lane >> 4, l16 = lane & 15;

  // patch DMA descriptors: piece j = wid + 4*i writes pixels 16j .. 16j+15, lane -> pixel
  // 16j + lane/4, physical slot lane & 3 (fetches logical slot (lane & 3) ^ g)
  int pv[P_PW], ps[P_PW];
#pragma unroll
  for (int i = 0; i < P_PW; ++i) {
    const int pix = (wid + 4 * i) * 16 + (lane >> 2);
    ps[i] = (lane & 3) ^ gsw((pix >> 2) & 3);
    pv[i] = -1;
    if (pix < PPIX) {
      const int ptt = pix / (QR * QC), r = pix - ptt * (QR * QC);
      const int pr = r / QC, pc = r - pr * QC;
      const int ti = t0 + ptt, hi = h0 - 1 + pr, wi = w0 - 1 + pc;
      if (ti < p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
        pv[i] = ((nclip * p.Ti + ti) * p.Hi + hi) * p.Wi + wi;
    }
  }
  // B DMA descriptors (conv_dma's swizzled 64-B rows)
  const int drow = lane >> 2;
  const int dq = (lane & 3) ^ gsw((drow >> 2) & 3);
  const __bf16* wrow[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int j = wid + 4 * i;
    wrow[i] = w + (size_t)(n0 + (j < NT ? j : 0) * 16 + drow) * p.Kp + 8 * dq;
  }

  const int Cin = p.Cin;
  auto issue_patch = [&](int c, int buf) {
    const int c0 = c * 32;
#pragma unroll
    for (int i = 0; i < P_PW; ++i) {
      const void* src = pv[i] >= 0 ? (const void*)(x + (size_t)(unsigned)pv[i] * Cin + c0 + 8 * ps[i]) : p.zero;
      char* dst = smem + buf * P_BYTES + (wid + 4 * i) * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  auto issue_b = [&](int s, int slot) {
    const int c = s / 9, tap = s - 9 * c;
    const int koff = tap * Cin + 32 * c;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const int j = wid + 4 * i;
      const void* src = j < NT ? (const void*)(wrow[i] + koff) : p.zero;
      char* dst = j < NT ? smem + B0 + slot * B_STAGE + j * 1024 : smem + JUNK;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  f32x4 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nc = Cin / 32, nk = 9 * nc;
  issue_patch(0, 0);
  issue_b(0, 0);
  if (nk > 1) issue_b(1, 1);

  // A fragment i of this lane: tile voxel m = 32*wid + 16*i + l16 -> patch pixel of tap (0,0)
  int abase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = wid * 32 + i * 16 + l16;
    abase[i] = ((m >> 6) * QR + ((m >> 3) & 7)) * QC + (m & 7);
  }
  const int b_off = B0 + l16 * 64 + (q ^ gsw(l16 >> 2)) * 16;

  for (int s = 0; s < nk; ++s) {
    const int c = s / 9, tap = s - 9 * c;
    if (s + 1 < nk) {
      if (tap == 1 && c + 1 < nc)  // the previous step issued B(s+1) and then the next patch
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_PW + P_PW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_PW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + 2 < nk) issue_b(s + 2, (s + 2) % S);
    if (tap == 0 && c + 1 < nc) issue_patch(c + 1, (c + 1) & 1);

    const char* pb = smem + (c & 1) * P_BYTES;
    const int kh = tap / 3, toff = kh * QC + (tap - 3 * kh);
    bf16x8 a[2], b[NT];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = abase[i] + toff;
      a[i] = *reinterpret_cast<const bf16x8*>(pb + pix * 64 + ((q ^ gsw((pix >> 2) & 3)) << 4));
    }
    const char* st = smem + (s % S) * B_STAGE + b_off;
#pragma unroll
    for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(st + j * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
  }

  // epilogue: accumulator acc[i][j] holds channels n0 + 16j + 4q .. +3 of tile voxel 32*wid + 16*i + l16
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const __bf16* res = reinterpret_cast<const __bf16*>(p.res);
  __bf16* y = reinterpret_cast<__bf16*>(p.y);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = wid * 32 + i * 16 + l16;
    const int to = t0 + (m >> 6), ho = h0 + ((m >> 3) & 7), wo = w0 + (m & 7);
    if (!(to < p.To && ho < p.Ho && wo < p.Wo)) continue;
    const size_t gm = (((size_t)nclip * p.To + to) * p.Ho + ho) * p.Wo + wo;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + j * 16 + 4 * q;
      if (n >= p.Cout) continue;
      const size_t o = gm * p.Cout + n;
      f32x4 v = acc[i][j];
      if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + n);
      if (res) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(res + o);
        v += f32x4{(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
      }
      if (p.relu) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.f);
      }
      *reinterpret_cast<bf16x4*>(y + o) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    }
  }
}

template <int NT>
hipError_t launch_patch(const ConvParams& p, hipStream_t s) {
  const int n_tiles = p.Cout / (16 * NT);
  const int tw = (p.Wo + PC - 1) / PC, th = (p.Ho + PR - 1) / PR, tt = (p.To + PT - 1) / PT;
  const long blocks = (long)p.N * tt * th * tw * n_tiles;
  hipLaunchKernelGGL((conv_patch_bf16<NT>), dim3((unsigned)blocks), dim3(256), 0, s, p, n_tiles, tw, th, tt);
  return hipGetLastError();
}

}  // namespace

bool patch_bf16_supported_v1(const ConvParams& p) {
  if (p.KT != 1) return false;
  if (!p.in_bf16 || !p.out_bf16 || p.stem || p.x2) return false;
  if (p.KT != 1 || p.KH != 3 || p.KW != 3 || p.st != 1 || p.sh != 1 || p.sw != 1) return false;
  if (p.pt != 0 || p.ph != 1 || p.pw != 1) return false;
  if (p.Cin % 32 || p.Cout % 16 || p.Kp != 9 * p.Cin) return false;
  if (p.To != p.Ti || p.Ho != p.Hi || p.Wo != p.Wi) return false;
  // voxel indices are int32 in the kernel
  if ((long)p.N * p.Ti * p.Hi * p.Wi >= (1L << 31) / 2) return false;
  return true;
}

hipError_t launch_patch_bf16_v1(const ConvParams& p, hipStream_t s) {
  const int n16 = p.Cout / 16;
  static const int force_nt = getenv("CLASFV_PATCH_NT") ? atoi(getenv("CLASFV_PATCH_NT")) : 0;  // A/B
  for (int nt : {10, 9, 8, 6, 5, 4}) {
    if (n16 % nt || (force_nt > 0 && nt != force_nt) || (force_nt <= 0 && nt == 10)) continue;
    switch (nt) {
      case 10: return launch_patch<10>(p, s);
      case 9: return launch_patch<9>(p, s);
      case 8: return launch_patch<8>(p, s);
      case 6: return launch_patch<6>(p, s);
      case 5: return launch_patch<5>(p, s);
      case 4: return launch_patch<4>(p, s);
    }
  }
  return hipErrorInvalidValue;
}
