// Fused Winograd F(4x4, 3x3) with WIDE output-channel blocks (conv_wino4w) for the stride-1 1x3x3 fp32
// convs: torchvision Conv2Plus1D's first conv (R(2+1)D-18 layer1-3 spatial halves, called through
// src/model/R2plus1D_18_MotionNet.py:31-37).
//
// Same arithmetic as conv_wino4 (winograd4.hip: Lavin's F(4,3) matrices, U = G g G^T formed in double
// on the host, v_mfma_f32_16x16x4_f32, the same K order), different block shape. conv_wino4 gives each
// block 48 output channels, so a 144-channel layer1 conv runs three blocks per tile group, each of
// which DMAs the same raw patch and transforms it again (FETCH 4.3x the input bytes, transform and DMA
// knock-outs 0.25 + 0.27 ms of a 2.1-ms launch, profiles/r03f_wino4_knockouts.txt). Here one block
// covers 16 NTN output channels (NTN = 9: all 144 of layer1, half of layer2's 288, a quarter of layer3's
// 576; NTN = 6 for 480): the patch is DMA'd and transformed once per tile group and every
// transformed value feeds NTN MFMAs instead of 3. The accumulators (9 Winograd elements x NTN x 4 =
// 324 registers at NTN = 9) need one wave per SIMD: 4-wave blocks, one per CU, 512 registers per lane.
// With no partner wave on the SIMD, U streams through a register ring UQ f32x4 loads deep (≈1800 MFMA
// cycles of L2 latency cover), the raw ring keeps two chunks in flight, and the epilogue's LDS planes
// are double-buffered (one barrier per 16 output channels).
//
// MFMA form D^T = U^T V^T (weights as the A operand): an accumulator lane holds 4 consecutive output
// channels of one tile, so the epilogue moves 16-B vectors through LDS in both directions (same
// products and accumulation order as the V U form: bit-identical to conv_wino4).
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "wino4_common.h"

namespace {

// Wide block of 16 NTN output channels: NV U values per lane per chunk (9 elements x 2 K steps x NTN),
// streamed as NU f32x4 loads (padded to a multiple of the ring depth UQ so every ring slot is a
// compile-time register in the unrolled chunk body).
template <int NTN>
struct W4W {
  static constexpr int NV = 18 * NTN;
  static constexpr int UQ = NTN == 9 ? 14 : 9;
  static constexpr int NU = (NV + 4 * UQ - 1) / (4 * UQ) * UQ;
};

// epilogue planes: [42][16 tiles][ZT], channel fastest (a lane's f32x4 = 4 channels of one tile);
// tile pitch 20 floats keeps the 8-lane groups of ds_write_b128 on distinct bank quads, plane pitch 324
// leaves the unit threads' ds_read_b128 at most 2-way conflicted (searched)
constexpr int W4W_ZT = 20;
constexpr int W4W_ZP = 16 * W4W_ZT + 4;
constexpr int W4W_ZBUF = 42 * W4W_ZP;  // floats per buffer (54,432 B)

// The f32 MFMA builtins accumulate in AGPRs (256 per lane); NTN = 9 needs 324 accumulator registers, and
// the compiler then moved accumulators between AGPRs and VGPRs around every MFMA (148 copies per chunk).
// So the N tiles past W4W_NTA accumulate in VGPRs through this statement. hipcc neither pads nor models
// an asm MFMA: the s_nop 1 covers a VALU-written B operand (the transform's), an accumulate chain of
// MFMAs needs no states, and the 12 states an 8-pass MFMA result needs before any other reader are
// padded after the chunk loop (w4w_drain). Its U operand comes from a builtin buffer load, which the
// compiler's vmcnt bookkeeping covers for any reader.
constexpr int W4W_NTA = 7;
__device__ inline void mfma_v(f32x4& c, float a, float b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ inline void w4w_drain() { asm volatile("s_nop 7\n\ts_nop 4" ::: "memory"); }

#ifdef CLASFV_KNOCKOUTS
// KO & 512 (tools/convbench diagnostic, not product): per block s_memrealtime (100 MHz) at entry, after
// the first chunk barrier, after the chunk loop and after the epilogue's stores completed, and the
// block's HW_ID / XCC_ID (profiles/r05c_wino4w_stamps.txt)
constexpr int W4W_NSTAMP = 16384;
__device__ unsigned long long g_w4w_stamps[W4W_NSTAMP][10];
#endif

template <int DPW>
constexpr int w4w_lds() {
  return W4Ring<DPW>::LDS > 2 * W4W_ZBUF * 4 ? W4Ring<DPW>::LDS : 2 * W4W_ZBUF * 4;
}

// C8: 8-channel-blocked output. DPW: DMA instructions per wave per chunk (W4Ring). KO: timing
// knock-outs for tools/convbench (0 in the product; results are wrong otherwise): 1 no transform,
// 2 no U loads in the loop, 4 no epilogue, 8 no DMAs in the loop, 128 the epilogue without its output
// stores, 256 the serial (unpipelined) epilogue order, 512 per-block phase stamps (diagnostic builds).
template <int NTN, bool C8, int DPW, int KO = 0, bool RELU = true>
__global__ __launch_bounds__(W4_THREADS) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv_wino4w(ConvParams p,
                                                                                                      W4Geo g) {
  using RG = W4Ring<DPW>;
  using WW = W4W<NTN>;
  constexpr int NR = RG::NR, STAGE = RG::STAGE, UQ = WW::UQ, NU = WW::NU;
  __shared__ __align__(16) char smem[w4w_lds<DPW>()];
  char* sink = smem + NR * STAGE;

#ifdef CLASFV_KNOCKOUTS
  unsigned long long st_[4] = {0, 0, 0, 0};
  if constexpr ((KO & 512) != 0) st_[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin * 4), 0x00020000);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int blk = xcd_swizzle4(blockIdx.x, gridDim.x);
  const int grp = fdiv(blk, g.fd_cob), cob = blk - grp * g.n_cob;
  const int rg = fdiv(grp, g.fd_gpr), gx = grp - rg * g.gpr;
  const int R0 = rg * g.TR, tx0 = gx * g.TC;
  const int H = p.Ho, W = p.Wo, C = p.Cin;
  const int nchunk = C >> 3;
  const int NT = g.TR * g.TC;

  // ---- LDS-DMA slot table (conv_wino4's): instruction j of this wave fills slots (wid + 4 j) * 64 +
  // lane of a stage; slot < RS: input channels 0..3 of a pixel, else 4..7
  unsigned d_off[6];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int ins = wid + W4_WAVES * j, s = ins * 64 + lane;
    unsigned off = 0x80000000u;
    if (ins < g.NI && s < 2 * g.RS) {
      const int hf = s >= g.RS ? 1 : 0, sl = s - hf * g.RS;
      const int seg = fdiv(sl, g.fd_ss), ss = sl - seg * g.SS;
      const int r = fdiv(ss, g.fd_rp), cs = ss - r * g.RP;
      const int m5 = cs / 5, k5 = cs - 5 * m5, c = 4 * m5 + k5;
      if (r < 6 && k5 < 4 && c < 4 * g.TC + 2) {
        const int R = R0 + seg, f = fdiv(R, g.fd_th), ty = R - f * g.TH;
        const int yy = 4 * ty - 1 + r, xx = 4 * tx0 - 1 + c;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = (((f * H + yy) * W + xx) * C + hf * 4) * 4;
      }
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int ins = wid + W4_WAVES * j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(ins < g.NI ? smem + stage * STAGE + ins * 1024 : sink), 16,
          d_off[j], k < nchunk ? k * 32 : 0, 0, 0);
    }
  };

  // ---- transform lane: tile t (MFMA column of V^T), channel pair k4 (K index) -- conv_wino4's
  const int rh = wid >> 1, ch = wid & 1;
  const int t = lane & 15, k4 = lane >> 4;
  const int tv = t < NT ? t : 0;
  const int tseg = fdiv(tv, g.fd_tc), tcol = tv - tseg * g.TC;
  const int lane_off = ((k4 >> 1) * g.RS + tseg * g.SS + rh * g.RP + 5 * tcol) * 16 + (k4 & 1) * 8;
  const int rp16 = g.RP * 16;
  auto transform = [&](int stage, f32x2 (&a)[3][3]) __attribute__((always_inline)) {
    if constexpr ((KO & 1) != 0) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) a[r][jj] = f32x2{(float)(lane + 3 * r + jj + stage), (float)(lane - jj)};
      return;
    }
    const char* base = smem + stage * STAGE + lane_off;
    auto body = [&](auto rh_c, auto ch_c) __attribute__((always_inline)) {
      constexpr int RH = decltype(rh_c)::value, CH = decltype(ch_c)::value;
      f32x2 tt[3][6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int co = (c + (c >> 2)) * 16;  // pixel columns 0..5 of the window -> slots 0,1,2,3,5,6
        f32x2 e[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) e[q] = *reinterpret_cast<const f32x2*>(base + q * rp16 + co);
        f32x2 t3[3];
        bt_rows<RH>(e, t3);
#pragma unroll
        for (int r = 0; r < 3; ++r) tt[r][c] = t3[r];
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) bt_cols<CH>(tt[r], a[r]);
    };
    switch (wid) {
      case 0: body(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}); break;
      case 1: body(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}); break;
      case 2: body(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}); break;
      default: body(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}); break;
    }
  };

  // ---- U operands: [cob][chunk][wave][NU][lane][4]; value m = 4 group + comp <-> MFMA (nt, r, ks, jj),
  // m = ((nt * 3 + r) * 2 + ks) * 3 + jj (m >= NV: zero pad)
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(reinterpret_cast<const float*>(p.w) + ((size_t)cob * nchunk * W4_WAVES + wid) * (NU * 256)),
      (short)0, nchunk * W4_WAVES * NU * 256 * 4, 0x00020000);
  // group G of the whole U stream (chunk G / NU); past the last chunk: re-reads of chunk 0 (counts only)
  auto load_u = [&](int k, int gi) __attribute__((always_inline)) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         ur, lane * 16, ((k < nchunk ? k : 0) * (W4_WAVES * NU * 256) + gi * 256) * 4, 0));
  };

  f32x4 acc[NTN][3][3];  // [nt][r][jj]: lane (tile l16, channels 4 q .. 4 q + 3 of N tile nt)
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) acc[nt][r][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 u[UQ];
  f32x2 a[3][3];

  // ---- prologue: raw(0), raw(1), then the first UQ U groups in flight
  issue_raw(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue_raw(1, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int gi = 0; gi < UQ; ++gi) u[gi] = load_u(0, gi);
  __builtin_amdgcn_sched_barrier(0);

  // chunk k in ring stage ph = k % NR. Every STEP chunks (a barrier) the stages of the STEP chunks
  // before k are refilled with raw(k+2) .. raw(k+NR-1). Per chunk every wave issues exactly NU U loads
  // (group gi + UQ right after the MFMAs that read group gi; NU is a multiple of UQ, so a group's ring
  // slot is gi % UQ in every chunk and the loop body is one chunk). Wait at a barrier: at most WAITN
  // VMEM ops outstanding -- fewer than are issued after raw(k+STEP-1) in any chunk (NR = 4: UQ on
  // chunk 0, 2 NU later; NR = 3: DPW + UQ on chunk 0, more later), so raw(k) .. raw(k+STEP-1) have
  // landed (conservative on later chunks, where the loads issued UQ groups back are done anyway).
  constexpr int WAITN = NR == 3 ? DPW + UQ : UQ;
  static_assert(WAITN <= 63, "vmcnt field");
  // (a do-while: Cin >= 8 gives at least one chunk, and a zero-trip path would merge zeroed
  // accumulators into the loop's, which made the compiler copy every accumulator to VGPRs at the exit)
  int k = 0;
#pragma unroll 1
  do {
    const int ph = k % NR;
    if (ph % RG::STEP == 0) {
      __builtin_amdgcn_s_waitcnt(vm_wait(WAITN));
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#ifdef CLASFV_KNOCKOUTS
      if constexpr ((KO & 512) != 0)
        if (k == 0) st_[1] = __builtin_amdgcn_s_memrealtime();
#endif
      if constexpr ((KO & 8) == 0) {
#pragma unroll
        for (int d = 2; d < NR; ++d) issue_raw(k + d, (ph + d) % NR);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    transform(ph, a);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int gi = 0; gi < NU; ++gi) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int m = 4 * gi + c;
        if (m < WW::NV) {
          const int jj = m % 3, ks = (m / 3) % 2, r = (m / 6) % 3, nt = m / 18;
          if (nt < W4W_NTA)
            acc[nt][r][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[gi % UQ][c], ks ? a[r][jj].y : a[r][jj].x,
                                                                  acc[nt][r][jj], 0, 0, 0);
          else
            mfma_v(acc[nt][r][jj], u[gi % UQ][c], ks ? a[r][jj].y : a[r][jj].x);
        }
      }
      if constexpr ((KO & 2) == 0) {
        const int gn = gi + UQ;  // the group this slot holds next: this chunk's, or the next chunk's
        u[gi % UQ] = gn < NU ? load_u(k, gn) : load_u(k + 1, gn - NU);
      }
    }
    // keep each reload right behind the MFMAs that read its slot (hoisted loads would need a register
    // per group in flight)
    // (the builtin MFMAs only: the asm ones of the N tiles past W4W_NTA come last in the chunk)
    constexpr int NB = (NTN < W4W_NTA ? NTN : W4W_NTA) * 18, FG = NB / 4, RM = NB % 4;
#pragma unroll
    for (int gi = 0; gi < NU; ++gi) {
      if (gi < FG)
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      else if (gi == FG && RM)
        __builtin_amdgcn_sched_group_barrier(0x008, RM, 0);
      if constexpr ((KO & 2) == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
  } while (++k < nchunk);
  if constexpr (NTN > W4W_NTA) w4w_drain();
  __builtin_amdgcn_s_waitcnt(vm_wait(0));  // past-the-end DMAs and U loads drained before LDS is reused
  __syncthreads();
#ifdef CLASFV_KNOCKOUTS
  if constexpr ((KO & 512) != 0) st_[2] = __builtin_amdgcn_s_memrealtime();
#endif

  if constexpr ((KO & 4) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) sum += acc[nt][r][jj][0] + acc[nt][r][jj][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  // ---- epilogue, per 16 output channels nt (Z double-buffered: one barrier per nt): wave (rh, ch)
  // stores the column partial sums of its rows i = 3 rh + r, P[i][b] = sum_j A^T[b][j] M[i][j] = E[e(b)]
  // + F[b] (ch 0: the distinct E = (m0+m1+m2, m1-m2, m1+m2), e(b) = 0, 1, 2, 1; ch 1: F = (m3+m4,
  // 2(m3-m4), 4(m3+m4), 8(m3-m4)+m5)); a thread then owns one unit (tile, 4 channels, column b) and
  // stores Y[a][b] = sum_i A^T[a][i] P[i][b], a = 0..3, 16 B per output pixel.
  float* Z0 = reinterpret_cast<float*>(smem);
  const int q = lane >> 4, l16 = lane & 15;
  const size_t plane = (size_t)p.N * p.To * H * W * 8;
  float* yout = reinterpret_cast<float*>(p.y);
  const int ub = tid & 3, ucq = (tid >> 2) & 3, utile = tid >> 4;
  const int useg = fdiv(utile, g.fd_tc), utc = utile - useg * g.TC;
  const int uR = R0 + useg, uf = fdiv(uR, g.fd_th), uty = uR - uf * g.TH;
  const int uxx = 4 * (tx0 + utc) + ub;
  const bool ulive = utile < NT && uxx < W;
  const int eb = ub == 3 ? 1 : ub;
  const int CO = p.Cout;
  auto write_planes = [&](int nt) __attribute__((always_inline)) {
    float* Z = Z0 + (nt & 1) * W4W_ZBUF;
    if (ch == 0) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const f32x4 m0 = acc[nt][r][0], m1 = acc[nt][r][1], m2 = acc[nt][r][2];
        f32x4* zp = reinterpret_cast<f32x4*>(Z + ((3 * rh + r) * 3) * W4W_ZP + l16 * W4W_ZT + 4 * q);
        zp[0] = m0 + m1 + m2;
        zp[W4W_ZP / 4] = psub4(m1, m2);
        zp[2 * W4W_ZP / 4] = m1 + m2;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const f32x4 m0 = acc[nt][r][0], m1 = acc[nt][r][1], m2 = acc[nt][r][2];
        f32x4* zp = reinterpret_cast<f32x4*>(Z + (18 + (3 * rh + r) * 4) * W4W_ZP + l16 * W4W_ZT + 4 * q);
        const f32x4 sm = m0 + m1, df = psub4(m0, m1);
        zp[0] = sm;
        zp[W4W_ZP / 4] = 2.f * df;
        zp[2 * W4W_ZP / 4] = 4.f * sm;
        zp[3 * W4W_ZP / 4] = 8.f * df + m2;
      }
    }
  };
  auto read_unit = [&](int nt, f32x4 (&P)[6]) __attribute__((always_inline)) {
    const float* Z = Z0 + (nt & 1) * W4W_ZBUF;
#pragma unroll
    for (int i = 0; i < 6; ++i)
      P[i] = *reinterpret_cast<const f32x4*>(Z + (i * 3 + eb) * W4W_ZP + utile * W4W_ZT + 4 * ucq) +
             *reinterpret_cast<const f32x4*>(Z + (18 + i * 4 + ub) * W4W_ZP + utile * W4W_ZT + 4 * ucq);
  };
  // output addresses: the thread's 4 pixel rows aa at N tile 0, then a uniform stride per N tile
  const int co0 = cob * NTN * 16 + 4 * ucq;
  const size_t upix = (size_t)(uf * H + 4 * uty) * W + uxx;
  float* ybase[4];
#pragma unroll
  for (int aa = 0; aa < 4; ++aa) {
    const size_t px = upix + (size_t)aa * W;
    ybase[aa] = yout + (C8 ? (size_t)(co0 >> 3) * plane + px * 8 + (co0 & 7) : px * CO + co0);
  }
  const size_t nt_step = C8 ? 2 * plane : 16;  // co + 16 per N tile
  // every N tile's bias, loaded before the first store: a bias load issued between the stores is the
  // wave's youngest vector-memory op, and its s_waitcnt vmcnt(0) waits for every store issued before
  // it (vmcnt retires in order) -- the epilogue then paid the store latency once per N tile
  // (profiles/r05d_wino4w_bias_preload.txt: epilogue 8.56 -> 7.85 us per layer1 block)
  f32x4 biasv[NTN];
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
    biasv[nt] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + co0 + nt * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
  auto store_unit = [&](int nt, const f32x4 (&P)[6]) __attribute__((always_inline)) {
    const f32x4 bias = biasv[nt];
    const f32x4 s12 = P[1] + P[2], d12 = psub4(P[1], P[2]), s34 = P[3] + P[4], d34 = psub4(P[3], P[4]);
    f32x4 y[4];
    y[0] = P[0] + s12 + s34;
    y[1] = d12 + 2.f * d34;
    y[2] = s12 + 4.f * s34;
    y[3] = d12 + 8.f * d34 + P[5];
#pragma unroll
    for (int aa = 0; aa < 4; ++aa) {
      if (4 * uty + aa >= H) break;  // partial tiles at the bottom edge (H % 4 != 0)
      f32x4 o = y[aa] + bias;
      if constexpr (RELU) {
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = relu1(o[c]);
      }
      float* dst = ybase[aa] + nt * nt_step;
      if constexpr ((KO & 128) != 0) {  // probe: no output stores
        if (o[0] == 1234.5f) *reinterpret_cast<f32x4*>(dst) = o;
      } else {
        *reinterpret_cast<f32x4*>(dst) = o;
      }
    }
  };
  if constexpr ((KO & 256) != 0) {
    // the first round-4 form (timing reference): write, barrier, read / transform / store per N tile
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      __builtin_amdgcn_sched_barrier(0);
      write_planes(nt);
      __syncthreads();
      if (ulive) {
        f32x4 P[6];
        read_unit(nt, P);
        store_unit(nt, P);
      }
    }
  } else {
    // software-pipelined: N tile nt's plane reads are issued, then N tile nt + 1's planes are written
    // into the other buffer (last read at nt - 1, before this iteration's barrier) while they are in
    // flight, then nt's output transform and stores run
    write_planes(0);
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      __builtin_amdgcn_sched_barrier(0);  // one N tile's accumulators at a time (no hoisted AGPR reads)
      __syncthreads();
      f32x4 P[6];
      if (ulive) read_unit(nt, P);
      if (nt + 1 < NTN) write_planes(nt + 1);
      if (ulive) store_unit(nt, P);
    }
  }
#ifdef CLASFV_KNOCKOUTS
  if constexpr ((KO & 512) != 0) {
    __builtin_amdgcn_s_waitcnt(0);  // the block's stores issued and complete
    __syncthreads();
    st_[3] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && blockIdx.x < W4W_NSTAMP) {
      unsigned long long* o = g_w4w_stamps[blockIdx.x];
      o[0] = st_[0], o[1] = st_[1], o[2] = st_[2], o[3] = st_[3];
      o[8] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
      o[9] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    }
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// conv_wino4r (round 5): conv_wino4w's tile groups, U values, products and accumulation order on 12
// waves per block -- three per SIMD instead of one. Wave (rh, ch, r) owns ONE row i = 3 rh + r of the
// quadrant (rh, ch): 3 Winograd elements x NTN N tiles = 108 accumulator registers at NTN = 9, so
// three waves fit a SIMD's 512 registers, and each SIMD interleaves three MFMA streams (the lone
// conv_wino4w wave issues back to back only where nothing else is in its stream: its chunk loop ran
// at ≈ 0.75 of the f32 MFMA rate, profiles/r05c_wino4w_stamps.txt). The epilogue exchanges three N
// tiles per round through three plane buffers (768 unit threads: one (tile, 4 channels, column b)
// unit of each), 3 rounds instead of 9 at NTN = 9. The cost: each wave reads its window rows of the
// raw patch itself (3x the transform's LDS reads, ≈ 1.2x its VALU: a row of B^T d is 1/3 of a
// quadrant's row transform).
constexpr int W4R_WAVES = 12;
constexpr int W4R_THREADS = 64 * W4R_WAVES;
constexpr int W4R_DPW = 2;  // DMA instructions per wave per ring stage (wino4_geometry: NI <= 24)
constexpr int W4R_STAGE = W4R_WAVES * W4R_DPW * 1024;
constexpr int W4R_NR = 4;  // raw ring stages (a barrier every NR / 2 chunks)
constexpr int W4R_NZ = 3;  // epilogue plane buffers = N tiles per epilogue round
constexpr int W4R_LDS = W4R_NZ * W4W_ZBUF * 4;  // 163,296 B
static_assert(W4R_LDS >= W4R_NR * W4R_STAGE + 1024 && W4R_LDS <= 160 * 1024, "ring and planes fit LDS");

// per wave and chunk: NV = 3 elements x 2 K steps x NTN U values, m = (nt * 2 + ks) * 3 + jj, as NU f32x4
// loads through a UQ-deep register ring
template <int NTN>
struct W4R {
  static constexpr int NV = 6 * NTN;
  static constexpr int UQ = NTN == 9 ? 7 : NTN == 5 ? 8 : 9;
  static constexpr int NU = (NV + 4 * UQ - 1) / (4 * UQ) * UQ;
};

// row R of bt_rows<RH> (the same expressions, so the same roundings)
template <int RH, int R>
__device__ inline f32x2 bt_row(const f32x2 (&e)[5]) {
  if constexpr (RH == 0) {
    if constexpr (R == 0) {
      return e[0] * 4.f - e[2] * 5.f + e[4];
    } else if constexpr (R == 1) {
      const f32x2 s = e[1] + e[2], u = e[3] + e[4];
      return u - s * 4.f;
    } else {
      const f32x2 d = e[1] - e[2], w = e[4] - e[3];
      return w + d * 4.f;
    }
  } else {
    if constexpr (R == 2) {
      return e[0] * 4.f - e[2] * 5.f + e[4];
    } else {
      const f32x2 x = e[3] - e[1], y = e[2] - e[0];
      if constexpr (R == 0)
        return x + y * 2.f;
      else
        return x - y * 2.f;
    }
  }
}

// KO (tools/convbench diagnostics, 0 in the product; results wrong otherwise): 1 no transform, 2 no U
// loads in the loop, 4 no epilogue, 8 no loop DMAs, 16 no chunk barriers, 128 no output stores, 512
// per-block phase stamps (as conv_wino4w's). NR: raw ring stages (4: a barrier every 2 chunks; 6: every 3)
template <int NTN, bool C8, int KO = 0, bool RELU = true, int NR = W4R_NR, int CPB = 1, bool NTS = false>
__global__ __launch_bounds__(W4R_THREADS) __attribute__((amdgpu_waves_per_eu(3, 3))) void conv_wino4r(ConvParams p,
                                                                                                       W4Geo g) {
  using WR = W4R<NTN>;
  constexpr int STAGE = W4R_STAGE, UQ = WR::UQ, NU = WR::NU, NV = WR::NV;
  constexpr int STEP = NR / 2;  // chunks per barrier: raw(k) .. raw(k + STEP - 1) land STEP chunks ahead
  static_assert(NR * STAGE + 1024 <= W4R_LDS, "ring fits the plane buffers' LDS");
  __shared__ __align__(16) char smem[W4R_LDS];
  char* sink = smem + NR * STAGE;

#ifdef CLASFV_KNOCKOUTS
  unsigned long long st_[4] = {0, 0, 0, 0};
  if constexpr ((KO & 512) != 0) st_[0] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef CLASFV_KNOCKOUTS
  // (convbench only) start stagger (W4Geo::stagger): blocks of equal work started together stay in lockstep, and all
  // 256 CUs then run their epilogues -- the output stores -- at once, reading nothing meanwhile
  // (profiles/r05ag_wino4r_epilogue_concurrency.txt); first-round blocks 8 j .. 8 j + 7 (one per XCD)
  // start (j % groups) stagger ticks apart, so the epilogues of different CUs fall in different phases
  if (g.stagger > 0 && blockIdx.x < 256) {
    const int sg = (blockIdx.x >> 3) % g.stagger_groups;
    if (sg) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), dt = (unsigned long long)sg * g.stagger;
      while (__builtin_amdgcn_s_memrealtime() - t0 < dt) __builtin_amdgcn_s_sleep(8);
    }
  }
#endif
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.N * p.Ti * p.Hi * p.Wi * p.Cin * 4), 0x00020000);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int blk = xcd_swizzle4(blockIdx.x, gridDim.x);
  const int grp = fdiv(blk, g.fd_cob), cob = blk - grp * g.n_cob;
  const int rg = fdiv(grp, g.fd_gpr), gx = grp - rg * g.gpr;
  const int R0 = rg * g.TR, tx0 = gx * g.TC;
  const int H = p.Ho, W = p.Wo, C = p.Cin;
  const int nchunk = C >> 3;
  const int NT = g.TR * g.TC;
  // wave (rh, ch, r) = wid / 6, (wid / 3) % 2, wid % 3
  const int wq = wid / 3, r = wid - 3 * wq, rh = wq >> 1, ch = wq & 1;

  // ---- LDS-DMA slot table (conv_wino4w's, over 12 waves): instruction j of this wave fills slots
  // (wid + 12 j) * 64 + lane of a stage
  unsigned d_off[W4R_DPW];
#pragma unroll
  for (int j = 0; j < W4R_DPW; ++j) {
    const int ins = wid + W4R_WAVES * j, s = ins * 64 + lane;
    unsigned off = 0x80000000u;
    if (ins < g.NI && s < 2 * g.RS) {
      const int hf = s >= g.RS ? 1 : 0, sl = s - hf * g.RS;
      const int seg = fdiv(sl, g.fd_ss), ss = sl - seg * g.SS;
      const int rr = fdiv(ss, g.fd_rp), cs = ss - rr * g.RP;
      const int m5 = cs / 5, k5 = cs - 5 * m5, c = 4 * m5 + k5;
      if (rr < 6 && k5 < 4 && c < 4 * g.TC + 2) {
        const int R = R0 + seg, f = fdiv(R, g.fd_th), ty = R - f * g.TH;
        const int yy = 4 * ty - 1 + rr, xx = 4 * tx0 - 1 + c;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = (((f * H + yy) * W + xx) * C + hf * 4) * 4;
      }
    }
    d_off[j] = off;
  }
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < W4R_DPW; ++j) {
      const int ins = wid + W4R_WAVES * j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(ins < g.NI ? smem + stage * STAGE + ins * 1024 : sink), 16,
          d_off[j], k < nchunk ? k * 32 : 0, 0, 0);
    }
  };

  // ---- transform lane: tile t, channel pair k4 (conv_wino4w's); this wave's row of B^T d B
  const int t = lane & 15, k4 = lane >> 4;
  const int tv = t < NT ? t : 0;
  const int tseg = fdiv(tv, g.fd_tc), tcol = tv - tseg * g.TC;
  const int lane_off = ((k4 >> 1) * g.RS + tseg * g.SS + rh * g.RP + 5 * tcol) * 16 + (k4 & 1) * 8;
  const int rp16 = g.RP * 16;
  auto transform = [&](int stage, f32x2 (&a)[3]) __attribute__((always_inline)) {
    if constexpr ((KO & 1) != 0) {
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) a[jj] = f32x2{(float)(lane + jj + stage), (float)(lane - jj)};
      return;
    }
    const char* base = smem + stage * STAGE + lane_off;
    auto body = [&](auto rh_c, auto ch_c, auto r_c) __attribute__((always_inline)) {
      constexpr int RH = decltype(rh_c)::value, CH = decltype(ch_c)::value, RR = decltype(r_c)::value;
      f32x2 tt[6];
      if constexpr (CPB == 0) {
        // software-pipelined: column c + 1's window reads are issued before column c's row transform,
        // so one LDS round trip is exposed per chunk instead of six (two columns' reads live at once)
        auto col_read = [&](int c, f32x2 (&e)[5]) __attribute__((always_inline)) {
          const int co = (c + (c >> 2)) * 16;
#pragma unroll
          for (int q = 0; q < 5; ++q) e[q] = *reinterpret_cast<const f32x2*>(base + q * rp16 + co);
        };
        f32x2 e0[5], e1[5];
        col_read(0, e0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 6; c += 2) {
          if (c + 1 < 6) col_read(c + 1, e1);
          tt[c] = bt_row<RH, RR>(e0);
          __builtin_amdgcn_sched_barrier(0);
          if (c + 2 < 6) col_read(c + 2, e0);
          tt[c + 1] = bt_row<RH, RR>(e1);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const int co = (c + (c >> 2)) * 16;  // pixel columns 0..5 of the window -> slots 0,1,2,3,5,6
          f32x2 e[5];
#pragma unroll
          for (int q = 0; q < 5; ++q) e[q] = *reinterpret_cast<const f32x2*>(base + q * rp16 + co);
          tt[c] = bt_row<RH, RR>(e);
          // CPB columns' window reads in flight at a time: 168 registers hold 108 accumulators and the
          // U ring (hoisting every column's reads spilled)
          if (c % CPB == CPB - 1) __builtin_amdgcn_sched_barrier(0);
        }
      }
      bt_cols<CH>(tt, a);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    switch (wid) {
      case 0: body(I0{}, I0{}, I0{}); break;
      case 1: body(I0{}, I0{}, I1{}); break;
      case 2: body(I0{}, I0{}, I2{}); break;
      case 3: body(I0{}, I1{}, I0{}); break;
      case 4: body(I0{}, I1{}, I1{}); break;
      case 5: body(I0{}, I1{}, I2{}); break;
      case 6: body(I1{}, I0{}, I0{}); break;
      case 7: body(I1{}, I0{}, I1{}); break;
      case 8: body(I1{}, I0{}, I2{}); break;
      case 9: body(I1{}, I1{}, I0{}); break;
      case 10: body(I1{}, I1{}, I1{}); break;
      default: body(I1{}, I1{}, I2{}); break;
    }
  };

  // ---- U operands: [cob][chunk][wave][NU][lane][4] (wino4r_transform_weights)
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(reinterpret_cast<const float*>(p.w) + ((size_t)cob * nchunk * W4R_WAVES + wid) * (NU * 256)),
      (short)0, nchunk * W4R_WAVES * NU * 256 * 4, 0x00020000);
  auto load_u = [&](int k, int gi) __attribute__((always_inline)) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         ur, lane * 16, ((k < nchunk ? k : 0) * (W4R_WAVES * NU * 256) + gi * 256) * 4, 0));
  };

  f32x4 acc[NTN][3];  // [nt][jj]: lane (tile l16, channels 4 q .. 4 q + 3 of N tile nt), element (i, 3 ch + jj)
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) acc[nt][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 u[UQ];
  f32x2 a[3];

#pragma unroll
  for (int d = 0; d < STEP; ++d) {
    issue_raw(d, d);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int gi = 0; gi < UQ; ++gi) u[gi] = load_u(0, gi);
  __builtin_amdgcn_sched_barrier(0);

  // the ring and wait rule of conv_wino4w at NR = 4: every 2 chunks a barrier, then raw(k + 2),
  // raw(k + 3) into the stages of chunks k - 2, k - 1; at most UQ VMEM ops outstanding at the wait
  // (the U loads issued after raw(k + 1) on chunk 0, 2 NU later) leaves raw(k), raw(k + 1) landed
  int k = 0;
#pragma unroll 1
  do {
    const int ph = k % NR;
    if (ph % STEP == 0) {
      __builtin_amdgcn_s_waitcnt(vm_wait(UQ));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((KO & 16) == 0) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#ifdef CLASFV_KNOCKOUTS
      if constexpr ((KO & 512) != 0)
        if (k == 0) st_[1] = __builtin_amdgcn_s_memrealtime();
#endif
      if constexpr ((KO & 8) == 0) {
#pragma unroll
        for (int d = NR - STEP; d < NR; ++d) issue_raw(k + d, (ph + d) % NR);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    transform(ph, a);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int gi = 0; gi < NU; ++gi) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int m = 4 * gi + c;
        if (m < NV) {
          const int jj = m % 3, ks = (m / 3) % 2, nt = m / 6;
          acc[nt][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[gi % UQ][c], ks ? a[jj].y : a[jj].x, acc[nt][jj], 0, 0, 0);
        }
      }
      if constexpr ((KO & 2) == 0) {
        const int gn = gi + UQ;
        u[gi % UQ] = gn < NU ? load_u(k, gn) : load_u(k + 1, gn - NU);
      }
    }
    constexpr int FG = NV / 4, RM = NV % 4;
#pragma unroll
    for (int gi = 0; gi < NU; ++gi) {
      if (gi < FG)
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      else if (gi == FG && RM)
        __builtin_amdgcn_sched_group_barrier(0x008, RM, 0);
      if constexpr ((KO & 2) == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
  } while (++k < nchunk);
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  __syncthreads();
#ifdef CLASFV_KNOCKOUTS
  if constexpr ((KO & 512) != 0) st_[2] = __builtin_amdgcn_s_memrealtime();
#endif

  if constexpr ((KO & 4) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) sum += acc[nt][jj][0] + acc[nt][jj][3];
    if (sum == 1234.5f) reinterpret_cast<float*>(p.y)[tid] = sum;
    return;
  }
  // ---- epilogue: conv_wino4w's planes and output transform, W4R_NZ N tiles per round: every wave
  // writes its row's planes of the round's N tiles into buffers 0..2, then thread (ug, unit) reads,
  // transforms and stores unit `unit` of N tile 3 round + ug
  float* Z0 = reinterpret_cast<float*>(smem);
  const int q = lane >> 4, l16 = lane & 15;
  const size_t plane = (size_t)p.N * p.To * H * W * 8;
  float* yout = reinterpret_cast<float*>(p.y);
  const int ug = tid >> 8, ut = tid & 255;
  const int ub = ut & 3, ucq = (ut >> 2) & 3, utile = ut >> 4;
  const int useg = fdiv(utile, g.fd_tc), utc = utile - useg * g.TC;
  const int uR = R0 + useg, uf = fdiv(uR, g.fd_th), uty = uR - uf * g.TH;
  const int uxx = 4 * (tx0 + utc) + ub;
  const bool ulive = utile < NT && uxx < W;
  const int eb = ub == 3 ? 1 : ub;
  const int CO = p.Cout;
  const int zrow = 3 * rh + r;
  auto write_planes = [&](int nt, int buf) __attribute__((always_inline)) {
    float* Z = Z0 + buf * W4W_ZBUF;
    const f32x4 m0 = acc[nt][0], m1 = acc[nt][1], m2 = acc[nt][2];
    if (ch == 0) {
      f32x4* zp = reinterpret_cast<f32x4*>(Z + (zrow * 3) * W4W_ZP + l16 * W4W_ZT + 4 * q);
      zp[0] = m0 + m1 + m2;
      zp[W4W_ZP / 4] = psub4(m1, m2);
      zp[2 * W4W_ZP / 4] = m1 + m2;
    } else {
      f32x4* zp = reinterpret_cast<f32x4*>(Z + (18 + zrow * 4) * W4W_ZP + l16 * W4W_ZT + 4 * q);
      const f32x4 sm = m0 + m1, df = psub4(m0, m1);
      zp[0] = sm;
      zp[W4W_ZP / 4] = 2.f * df;
      zp[2 * W4W_ZP / 4] = 4.f * sm;
      zp[3 * W4W_ZP / 4] = 8.f * df + m2;
    }
  };
  auto read_unit = [&](int buf, f32x4 (&P)[6]) __attribute__((always_inline)) {
    const float* Z = Z0 + buf * W4W_ZBUF;
#pragma unroll
    for (int i = 0; i < 6; ++i)
      P[i] = *reinterpret_cast<const f32x4*>(Z + (i * 3 + eb) * W4W_ZP + utile * W4W_ZT + 4 * ucq) +
             *reinterpret_cast<const f32x4*>(Z + (18 + i * 4 + ub) * W4W_ZP + utile * W4W_ZT + 4 * ucq);
  };
  const int co0 = cob * NTN * 16 + 4 * ucq;
  const size_t upix = (size_t)(uf * H + 4 * uty) * W + uxx;
  float* ybase[4];
#pragma unroll
  for (int aa = 0; aa < 4; ++aa) {
    const size_t px = upix + (size_t)aa * W;
    ybase[aa] = yout + (C8 ? (size_t)(co0 >> 3) * plane + px * 8 + (co0 & 7) : px * CO + co0);
  }
  const size_t nt_step = C8 ? 2 * plane : 16;
  constexpr int NRND = (NTN + W4R_NZ - 1) / W4R_NZ;
  // this thread's N tiles' bias, loaded before the first store (conv_wino4w's reason)
  f32x4 biasv[NRND];
#pragma unroll
  for (int rd = 0; rd < NRND; ++rd) {
    const int nt = W4R_NZ * rd + ug;
    biasv[rd] = p.bias && nt < NTN ? *reinterpret_cast<const f32x4*>(p.bias + co0 + nt * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto store_unit = [&](int nt, const f32x4& bias, const f32x4 (&P)[6]) __attribute__((always_inline)) {
    const f32x4 s12 = P[1] + P[2], d12 = psub4(P[1], P[2]), s34 = P[3] + P[4], d34 = psub4(P[3], P[4]);
    f32x4 y[4];
    y[0] = P[0] + s12 + s34;
    y[1] = d12 + 2.f * d34;
    y[2] = s12 + 4.f * s34;
    y[3] = d12 + 8.f * d34 + P[5];
#pragma unroll
    for (int aa = 0; aa < 4; ++aa) {
      if (4 * uty + aa >= H) break;
      f32x4 o = y[aa] + bias;
      if constexpr (RELU) {
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = relu1(o[c]);
      }
      float* dst = ybase[aa] + nt * nt_step;
      if constexpr ((KO & 128) != 0) {
        if (o[0] == 1234.5f) *reinterpret_cast<f32x4*>(dst) = o;
      } else if constexpr (NTS || (KO & 2048) != 0) {  // non-temporal output stores (the product form)
        __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(dst));
      } else {
        *reinterpret_cast<f32x4*>(dst) = o;
      }
    }
  };
#pragma unroll
  for (int b = 0; b < W4R_NZ; ++b)
    if (b < NTN) write_planes(b, b);
#pragma unroll
  for (int rd = 0; rd < NRND; ++rd) {
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    const int nt_u = W4R_NZ * rd + ug;
    const bool live = ulive && nt_u < NTN;
    f32x4 P[6];
    if (live) read_unit(ug, P);
    if (rd + 1 < NRND) {
      __syncthreads();
#pragma unroll
      for (int b = 0; b < W4R_NZ; ++b)
        if (W4R_NZ * (rd + 1) + b < NTN) write_planes(W4R_NZ * (rd + 1) + b, b);
    }
    if (live) store_unit(nt_u, biasv[rd], P);
  }
#ifdef CLASFV_KNOCKOUTS
  if constexpr ((KO & 512) != 0) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    st_[3] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && blockIdx.x < W4W_NSTAMP) {
      unsigned long long* o = g_w4w_stamps[blockIdx.x];
      o[0] = st_[0], o[1] = st_[1], o[2] = st_[2], o[3] = st_[3];
      o[8] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
      o[9] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
  }
#endif
}

template <int NTN, int KO = 0, int NR = W4R_NR, int CPB = 1>
hipError_t launch_w4r(const ConvParams& p, const W4Geo& g, int n_blocks, hipStream_t s) {
  const dim3 grid(n_blocks), block(W4R_THREADS);
  // non-temporal output stores unless CLASFV_VARIANT_W4R_CACHED_STORES (the ReLU / C8 forms the forward
  // runs): the 144-channel mid tensor is streamed past L2 / MALL, and both this kernel and the temporal
  // Winograd that reads it next run faster (profiles/r05ab_w4r_nt_stores_ab.txt: wino4r 9.11 -> 9.05,
  // winot 5.46 -> 5.38 ms per forward, step 21.57 -> 21.38 ms)
  if (!(p.vflags & CLASFV_VARIANT_W4R_CACHED_STORES)) {
    if (p.y_c8 && p.relu) {
      hipLaunchKernelGGL((conv_wino4r<NTN, true, KO, true, NR, CPB, true>), grid, block, 0, s, p, g);
      return hipGetLastError();
    }
    if (p.relu) {
      hipLaunchKernelGGL((conv_wino4r<NTN, false, KO, true, NR, CPB, true>), grid, block, 0, s, p, g);
      return hipGetLastError();
    }
  }
  if (p.y_c8 && p.relu)
    hipLaunchKernelGGL((conv_wino4r<NTN, true, KO, true, NR, CPB>), grid, block, 0, s, p, g);
  else if (p.relu)
    hipLaunchKernelGGL((conv_wino4r<NTN, false, KO, true, NR, CPB>), grid, block, 0, s, p, g);
  else if (p.y_c8)
    hipLaunchKernelGGL((conv_wino4r<NTN, true, KO, false, NR, CPB>), grid, block, 0, s, p, g);
  else
    hipLaunchKernelGGL((conv_wino4r<NTN, false, KO, false, NR, CPB>), grid, block, 0, s, p, g);
  return hipGetLastError();
}

// tile groups: the most tiles per group (16 fills every MFMA row), then the widest, among column
// widths >= W4W_FILL (56x56 maps: 8 x 2 tiles, 28x28: 16 x 1)
// (profiles/r04_wino4w_fill16.txt)
constexpr int W4W_FILL = 1;

// NTN for a Cout: the widest of 9, 6 N tiles dividing it (0: none). NTN = 5 (layer2's 240 channels)
// compiles but ran 0.785 vs conv_wino4's 0.754 ms (r04b): the 80-channel block pays the one-wave-per-SIMD
// serialisation without enough reuse to win it back, so conv_wino4 keeps that conv.
int wino4w_ntn(int cout) {
  if (cout % 16) return 0;
  for (int n : {9, 6})
    if ((cout / 16) % n == 0) return n;
  return 0;
}

template <int NTN, int DPW, int KO = 0>
hipError_t launch_w4w(const ConvParams& p, const W4Geo& g, int n_blocks, hipStream_t s) {
  const dim3 grid(n_blocks), block(W4_THREADS);
  // every Conv2Plus1D spatial half is followed by BN + ReLU: the ReLU form is the one that runs
  if (p.y_c8 && p.relu)
    hipLaunchKernelGGL((conv_wino4w<NTN, true, DPW, KO, true>), grid, block, 0, s, p, g);
  else if (p.relu)
    hipLaunchKernelGGL((conv_wino4w<NTN, false, DPW, KO, true>), grid, block, 0, s, p, g);
  else if (p.y_c8)
    hipLaunchKernelGGL((conv_wino4w<NTN, true, DPW, KO, false>), grid, block, 0, s, p, g);
  else
    hipLaunchKernelGGL((conv_wino4w<NTN, false, DPW, KO, false>), grid, block, 0, s, p, g);
  return hipGetLastError();
}

template <int NTN, int KO = 0>
hipError_t launch_w4w_dpw(const ConvParams& p, const W4Geo& g, int n_blocks, hipStream_t s) {
  const int dpw = (g.NI + W4_WAVES - 1) / W4_WAVES;
  return dpw <= 4 ? launch_w4w<NTN, 4, KO>(p, g, n_blocks, s)
                  : dpw == 5 ? launch_w4w<NTN, 5, KO>(p, g, n_blocks, s) : launch_w4w<NTN, 6, KO>(p, g, n_blocks, s);
}

}  // namespace

bool wino4w_supported(const ConvParams& p) {
  W4Geo g;
  int nb;
  const int ntn = wino4w_ntn(p.Cout);
  return ntn && !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && !p.res && p.KT == 1 && p.KH == 3 && p.KW == 3 &&
         p.sh == 1 && p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Ho == p.Hi &&
         p.Wo == p.Wi && p.To == p.Ti &&
         (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31) &&
         wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL);
}

// p.w: wino4w_transform_weights' layout for this Cout's NTN.
hipError_t launch_wino4w(const ConvParams& p, hipStream_t s) {
  if (!wino4w_supported(p)) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  const int ntn = wino4w_ntn(p.Cout);
  wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL);
  return ntn == 9 ? launch_w4w_dpw<9>(p, g, nb, s) : launch_w4w_dpw<6>(p, g, nb, s);
}

// Every block issues 16 MFMA rows (tiles, the group's padding included) x 36 elements x Cin x 16 NTN.
double wino4w_exec_gflop(const ConvParams& p) {
  W4Geo g;
  int nb;
  const int ntn = wino4w_ntn(p.Cout);
  return ntn && wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL) ? 2.0 * nb * 16.0 * 36.0 * p.Cin * 16.0 * ntn * 1e-9 : 0.0;
}

// Floats of wino4w_transform_weights' output for a cin_p x cout_p conv (0: no wide block fits).
size_t wino4w_weight_floats(int cin_p, int cout_p) {
  const int ntn = wino4w_ntn(cout_p);
  if (!ntn) return 0;
  const int nu = ntn == 9 ? W4W<9>::NU : W4W<6>::NU;
  return (size_t)(cout_p / (16 * ntn)) * (cin_p / 8) * W4_WAVES * nu * 256;
}

// U[cout_p/(16 NTN)][cin_p/8][4 waves][NU][64 lane][4] from folded weights w[cout][cin][3][3] (double):
// wave = (rh, ch) = (w / 2, w % 2), lane = k4 * 16 + n, value m = 4 group + comp = ((nt * 3 + r) * 2 +
// ks) * 3 + jj (m >= 18 NTN: zero): element (3 rh + r, 3 ch + jj) of G g G^T for input channel chunk * 8
// + 2 k4 + ks and output channel cob * 16 NTN + nt * 16 + n.
void wino4w_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  const int ntn = wino4w_ntn(cout_p);
  const int nu = ntn == 9 ? W4W<9>::NU : W4W<6>::NU;
  const int nch = cin_p / 8, cw = 16 * ntn;
  const size_t total = wino4w_weight_floats(cin_p, cout_p);
  for (size_t i = 0; i < total; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* gw = w + ((size_t)o * cin + c) * 9;
      double tmp[6][3];
      for (int i = 0; i < 6; ++i)
        for (int v = 0; v < 3; ++v) tmp[i][v] = G[i][0] * gw[0 * 3 + v] + G[i][1] * gw[1 * 3 + v] + G[i][2] * gw[2 * 3 + v];
      const int cob = o / cw, nt = (o % cw) / 16, n = o % 16;
      const int chunk = c / 8, k4 = (c % 8) / 2, ks = c % 2;
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          const double uu = tmp[i][0] * G[j][0] + tmp[i][1] * G[j][1] + tmp[i][2] * G[j][2];
          const int wv = (i / 3) * 2 + j / 3, r = i % 3, jj = j % 3;
          const int m = ((nt * 3 + r) * 2 + ks) * 3 + jj, gi = m / 4, comp = m % 4;
          U[((((((size_t)cob * nch + chunk) * W4_WAVES + wv) * nu + gi) * 64) + k4 * 16 + n) * 4 + comp] = (float)uu;
        }
    }
}

// NTN of conv_wino4r for a Cout: the widest of 9, 6 N tiles dividing it (0: none). NTN = 5 (layer2's
// 240-channel conv) compiles (W4R<5>) but ran 0.747 vs conv_wino4's 0.723 ms
// (profiles/r05o_wino4r_ntn5.txt): conv_wino4 keeps that conv.
int wino4r_ntn(int cout) {
  if (cout % 16) return 0;
  for (int n : {9, 6})
    if ((cout / 16) % n == 0) return n;
  return 0;
}

static int w4r_nu(int ntn) { return ntn == 9 ? W4R<9>::NU : ntn == 6 ? W4R<6>::NU : W4R<5>::NU; }

bool wino4r_supported(const ConvParams& p) {
  W4Geo g;
  int nb;
  const int ntn = wino4r_ntn(p.Cout);
  return ntn && !p.in_bf16 && !p.out_bf16 && !p.stem && !p.x2 && !p.res && p.KT == 1 && p.KH == 3 && p.KW == 3 &&
         p.sh == 1 && p.sw == 1 && p.st == 1 && p.ph == 1 && p.pw == 1 && p.pt == 0 && p.Ho == p.Hi &&
         p.Wo == p.Wi && p.To == p.Ti &&
         (size_t)p.N * p.To * p.Ho * p.Wo * (p.Cin > p.Cout ? p.Cin : p.Cout) < ((size_t)1 << 31) &&
         wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL);
}

// conv_wino4r (12 row waves per block) on conv_wino4w's tile groups; p.w: wino4r_transform_weights' layout.
hipError_t launch_wino4r(const ConvParams& p, hipStream_t s) {
  if (!wino4r_supported(p)) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  const int ntn = wino4r_ntn(p.Cout);
  wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL);
  return ntn == 9 ? launch_w4r<9>(p, g, nb, s) : launch_w4r<6>(p, g, nb, s);
}

double wino4r_exec_gflop(const ConvParams& p) {
  W4Geo g;
  int nb;
  const int ntn = wino4r_ntn(p.Cout);
  return ntn && wino4_geometry(p, &g, &nb, 16 * ntn, W4W_FILL) ? 2.0 * nb * 16.0 * 36.0 * p.Cin * 16.0 * ntn * 1e-9 : 0.0;
}

size_t wino4r_weight_floats(int cin_p, int cout_p) {
  const int ntn = wino4r_ntn(cout_p);
  if (!ntn) return 0;
  return (size_t)(cout_p / (16 * ntn)) * (cin_p / 8) * W4R_WAVES * w4r_nu(ntn) * 256;
}

// U[cout_p/(16 NTN)][cin_p/8][12 waves][NU][64 lane][4]: wave (rh, ch, r) = (w / 6, (w / 3) % 2, w % 3),
// lane = k4 * 16 + n, value m = 4 group + comp = (nt * 2 + ks) * 3 + jj (m >= 6 NTN: zero): element
// (3 rh + r, 3 ch + jj) of G g G^T (conv_wino4w's values, double on the host) for input channel
// chunk * 8 + 2 k4 + ks and output channel cob * 16 NTN + nt * 16 + n.
void wino4r_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U) {
  static const double G[6][3] = {{1.0 / 4, 0, 0},
                                 {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                 {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                 {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                 {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                 {0, 0, 1}};
  const int ntn = wino4r_ntn(cout_p);
  const int nu = w4r_nu(ntn);
  const int nch = cin_p / 8, cw = 16 * ntn;
  const size_t total = wino4r_weight_floats(cin_p, cout_p);
  for (size_t i = 0; i < total; ++i) U[i] = 0.f;
  for (int o = 0; o < cout; ++o)
    for (int c = 0; c < cin; ++c) {
      const double* gw = w + ((size_t)o * cin + c) * 9;
      double tmp[6][3];
      for (int i = 0; i < 6; ++i)
        for (int v = 0; v < 3; ++v) tmp[i][v] = G[i][0] * gw[0 * 3 + v] + G[i][1] * gw[1 * 3 + v] + G[i][2] * gw[2 * 3 + v];
      const int cob = o / cw, nt = (o % cw) / 16, n = o % 16;
      const int chunk = c / 8, k4 = (c % 8) / 2, ks = c % 2;
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          const double uu = tmp[i][0] * G[j][0] + tmp[i][1] * G[j][1] + tmp[i][2] * G[j][2];
          const int wv = ((i / 3) * 2 + j / 3) * 3 + i % 3, jj = j % 3;
          const int m = (nt * 2 + ks) * 3 + jj, gi = m / 4, comp = m % 4;
          U[((((((size_t)cob * nch + chunk) * W4R_WAVES + wv) * nu + gi) * 64) + k4 * 16 + n) * 4 + comp] = (float)uu;
        }
    }
}

#ifdef CLASFV_KNOCKOUTS
void wino4w_stamps(unsigned long long* out, int n) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w4w_stamps), sizeof(unsigned long long) * 10 * (n < W4W_NSTAMP ? n : W4W_NSTAMP));
}
// tools/convbench: conv_wino4w timing knock-outs (KO bits above; 1024: conv_wino4's tile-group rule).
hipError_t launch_wino4w_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (!wino4w_supported(p) || wino4w_ntn(p.Cout) != 9) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  // ko 1024 + bits: the widest-TC tile groups (conv_wino4's shape rule) instead of 16-tile groups;
  // 2048 + bits: 16-tile groups down to one tile column
  wino4_geometry(p, &g, &nb, 144, (ko & 1024) ? 0 : (ko & 2048) ? 1 : W4W_FILL);
  ko &= ~3072;
  switch (ko) {
    case 1: return launch_w4w_dpw<9, 1>(p, g, nb, s);
    case 2: return launch_w4w_dpw<9, 2>(p, g, nb, s);
    case 4: return launch_w4w_dpw<9, 4>(p, g, nb, s);
    case 8: return launch_w4w_dpw<9, 8>(p, g, nb, s);
    case 15: return launch_w4w_dpw<9, 15>(p, g, nb, s);
    case 128: return launch_w4w_dpw<9, 128>(p, g, nb, s);
    case 256: return launch_w4w_dpw<9, 256>(p, g, nb, s);
    case 512: return launch_w4w_dpw<9, 512>(p, g, nb, s);
    default: return launch_w4w_dpw<9>(p, g, nb, s);
  }
}
// tools/convbench: conv_wino4r diagnostics (KO bits of conv_wino4r; 64: the 6-stage ring), NTN = 9 only
hipError_t launch_wino4r_ko(const ConvParams& p, hipStream_t s, int ko) {
  if (!wino4w_supported(p) || wino4w_ntn(p.Cout) != 9) return hipErrorInvalidValue;
  W4Geo g;
  int nb;
  wino4_geometry(p, &g, &nb, 144, W4W_FILL);
  if (const char* e = getenv("CB_W4R_STAGGER")) sscanf(e, "%d,%d", &g.stagger, &g.stagger_groups);  // ticks,groups
  switch (ko) {
    case 1: return launch_w4r<9, 1>(p, g, nb, s);
    case 2: return launch_w4r<9, 2>(p, g, nb, s);
    case 8: return launch_w4r<9, 8>(p, g, nb, s);
    case 16: return launch_w4r<9, 16>(p, g, nb, s);
    case 31: return launch_w4r<9, 31>(p, g, nb, s);
    case 4: return launch_w4r<9, 4>(p, g, nb, s);
    case 128: return launch_w4r<9, 128>(p, g, nb, s);
    case 512: return launch_w4r<9, 512>(p, g, nb, s);
    case 64: return launch_w4r<9, 0, 6>(p, g, nb, s);     // 6-stage ring, a barrier every 3 chunks
    case 32: return launch_w4r<9, 0, 4, 2>(p, g, nb, s);  // 2 window columns' LDS reads in flight
    case 96: return launch_w4r<9, 0, 4, 3>(p, g, nb, s);  // 3
    case 160: return launch_w4r<9, 0, 4, 0>(p, g, nb, s);  // software-pipelined column reads
    case 2048: return launch_w4r<9, 2048>(p, g, nb, s);    // non-temporal output stores
    case 576: return launch_w4r<9, 512, 6>(p, g, nb, s);  // the same with stamps
    default: return launch_w4r<9>(p, g, nb, s);
  }
}
// the wino4r image of a conv_wino4w image (a permutation: the same U values in wino4r's order)
void wino4r_from_wino4w(const float* Uw, int cin_p, int cout_p, float* Ur) {
  const int ntn = wino4w_ntn(cout_p);
  const int nuw = ntn == 9 ? W4W<9>::NU : W4W<6>::NU, nur = ntn == 9 ? W4R<9>::NU : W4R<6>::NU;
  const int nch = cin_p / 8, ncob = cout_p / (16 * ntn);
  for (size_t i = 0; i < wino4r_weight_floats(cin_p, cout_p); ++i) Ur[i] = 0.f;
  for (int cob = 0; cob < ncob; ++cob)
    for (int ck = 0; ck < nch; ++ck)
      for (int wv = 0; wv < 4; ++wv)
        for (int r = 0; r < 3; ++r)
          for (int nt = 0; nt < ntn; ++nt)
            for (int ks = 0; ks < 2; ++ks)
              for (int jj = 0; jj < 3; ++jj) {
                const int mw = ((nt * 3 + r) * 2 + ks) * 3 + jj, mr = (nt * 2 + ks) * 3 + jj;
                for (int l = 0; l < 64; ++l)
                  Ur[(((((size_t)cob * nch + ck) * W4R_WAVES + wv * 3 + r) * nur + mr / 4) * 64 + l) * 4 + mr % 4] =
                      Uw[(((((size_t)cob * nch + ck) * 4 + wv) * nuw + mw / 4) * 64 + l) * 4 + mw % 4];
              }
}
#endif
