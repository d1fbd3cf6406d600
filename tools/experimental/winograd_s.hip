// Warp-specialised persistent Winograd F(2x2, 3x3) for the widest stride-1 1x3x3 fp32 convs (R(2+1)D-18
// layer1 at 32x112x112 clips: 56x56 maps; layer2 of 224x224 clips). Same op, arithmetic, U layout,
// accumulation order and epilogue arithmetic as conv_wino_q (winograd2.hip), so the outputs are bit for
// bit the same; what changes is who does what:
//
//  * one 512-thread block per CU, persistent over a contiguous run of work items (item = 2 patches of
//    8x8 output pixels = 32 tiles x 48 output channels; the co groups of a patch pair are consecutive
//    items, so their raw input is re-read from the CU's own caches);
//  * waves 0-3 are CONSUMERS: wave i owns the Winograd row e = 4i..4i+3 and only issues MFMAs (V
//    operands from LDS one chunk ahead, U operands from L2 two chunks ahead); waves 4-7 are PRODUCERS:
//    LDS-DMA of the raw 10x10-pixel patches four chunks ahead, the input transform two chunks ahead,
//    and the previous item's epilogue (Z exchange read, output transform, bias / residual / ReLU,
//    stores). Consumer i and producer i + 4 share a SIMD, so the transform / epilogue VALU and LDS work
//    runs in the issue slots beside the consumer's MFMA stream instead of in line with it;
//  * the chunk stream runs across item boundaries: the consumer hands an item's accumulators over as
//    Z rows in LDS and starts the next item's MFMAs at once; no per-item prologue or epilogue stalls
//    the matrix pipe (conv_wino_q: 6 % + 10 % of its time).
//
// One s_barrier per 8-channel chunk (all 8 waves). Interval s (chunk position s of the block's stream):
//   producers: raw(s+2) landed -> barrier -> DMA raw(s+4) into ring stage (s+4)%3 -> transform raw(s+2)
//              into V stage (s+2)%3 -> [first chunk of an item] epilogue of the previous item from Z;
//   consumers: U(s), A(s) in registers -> barrier -> read A(s+1) from V stage (s+1)%3 -> 48 MFMAs of
//              chunk s -> load U(s+2) into the U registers chunk s has just consumed (2-way rotation,
//              so every register index is a compile-time constant for even chunk counts) ->
//              [last chunk of an item] Z rows to LDS.
//   The producers issue an item's epilogue stores at the start of an interval, before its DMAs, so a
//   uniform vmcnt(2) at the next interval covers both (store counts differ between producer waves).
#include "common.h"

// (declarations the product header no longer carries: this kernel is an experiment, tools/ only)
bool winos_supported(const ConvParams& p);
hipError_t launch_winos(const ConvParams& p, hipStream_t s);

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ inline void dma16s(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

constexpr int S_BT = 32;                   // tiles per item
constexpr int S_V = 16 * S_BT * 32;        // V stage: 16 e x 32 tiles x 8 channels x 4 B = 16 KB
constexpr int S_SIDE = 10, S_PIX = 100;    // 10x10-pixel input patch of 4x4 tiles
constexpr int S_PSTRIDE = S_PIX + 1;       // odd pixel stride between the two patches of a stage
constexpr int S_SLOTS = 2 * S_PSTRIDE * 2; // 16-B DMA slots per chunk (8 channels = 2 x 16 B per pixel)
constexpr int S_DPW = 2;                   // DMAs per producer wave per chunk (4 waves x 2 x 64 >= 404)
constexpr int S_RAW = 4 * S_DPW * 1024;    // raw stage: 8 KB
constexpr int S_Z = 4 * S_BT * 48 * 8;     // Z rows: 4 i x 32 tiles x 48 co x f32x2 = 48 KB
constexpr int S_LDS = 3 * S_RAW + 3 * S_V + S_Z;  // 120 KB: one block per CU
static_assert(4 * S_DPW * 64 >= S_SLOTS, "raw slots");

struct Item {
  int pair, n0;  // patch pair index (patches 2 pair, 2 pair + 1) and first output channel
};

#ifdef CLASFV_KNOCKOUTS
// diagnostic stamps (tools/convbench.hip, VAR bit 2): per block < 8, per role, cycles spent in the
// per-chunk wait + barrier and in total (lane 0 of waves 0 and 4)
__device__ unsigned long long g_wstamps[8][2][2];
#endif

// EPI: bit 0 residual add, bit 1 ReLU; C8: 8-channel-blocked output (see conv_wino_q). VAR (timing
// experiments only, 0 in the product): bit 0 consumer priority, bit 1 no producer priority, bit 2 stamps;
// knock-outs (wrong results, timing only): bit 3 no epilogue, bit 4 no transform, bit 5 no MFMAs,
// bit 6 no U loads in the chunk loop (stale U registers).
template <int NCH, int EPI, bool C8, int VAR = 0>
__global__ __launch_bounds__(512) void conv_wino_s(ConvParams p, int n_co, int n_patches, int n_pairs,
                                                    FastDiv fd_co, FastDiv fd_frame, FastDiv fd_px) {
  static_assert(NCH >= 4, "the DMA stream runs 4 chunks ahead within one item boundary");
  extern __shared__ __align__(16) char smem[];
  char* raw = smem;
  char* vbuf = smem + 3 * S_RAW;
  f32x2* zs = reinterpret_cast<f32x2*>(smem + 3 * S_RAW + 3 * S_V);

  const float* x = reinterpret_cast<const float*>(p.x);
  const float* U = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wid < 4;
  const int rw = wid & 3;  // row / producer wave index
  const int H = p.Ho, W = p.Wo, C = p.Cin, CO = p.Cout;
  const int PY = H / 8, PX = W / 8;

  // contiguous run of patch pairs for this block; its items are (pair, co group) with co fastest
  const int G = gridDim.x, b = blockIdx.x;
  const int q0 = n_pairs / G, r0 = n_pairs - q0 * G;
  const int pair_lo = b * q0 + min(b, r0);
  const int n_items = (q0 + (b < r0 ? 1 : 0)) * n_co;
  auto item_of = [&](int t) __attribute__((always_inline)) {
    const int pi = fdiv(t, fd_co);
    return Item{pair_lo + pi, (t - pi * n_co) * 48};
  };

  // the producers' latency chains, not the consumers' MFMA stream, set the interval length
  // (tools/gpu_winos_b.sh stamps): the producers get the issue priority
  if ((VAR & 1) && consumer) __builtin_amdgcn_s_setprio(1);
  if (!(VAR & 2) && !consumer) __builtin_amdgcn_s_setprio(1);
  unsigned long long st_wait = 0, st_t0 = 0;
  if constexpr ((VAR & 4) != 0) st_t0 = __builtin_amdgcn_s_memtime();
  auto stamp_wait = [&](unsigned long long a) __attribute__((always_inline)) {
    if constexpr ((VAR & 4) != 0) st_wait += __builtin_amdgcn_s_memtime() - a;
  };
  auto now = [&]() __attribute__((always_inline)) -> unsigned long long {
    if constexpr ((VAR & 4) != 0) return __builtin_amdgcn_s_memtime();
    return 0;
  };

  // ---- consumer state --------------------------------------------------------------------------
  const int q = lane >> 4, l16 = lane & 15;
  const float* ub0 = U + (((size_t)rw * CO + l16) * 4 + q) * 8;  // + n0 * 32 + chunk * 4 * CO * 32
  f32x4 uu[2][3][2];
  f32x4 aa[2][4];
  f32x4 acc[4][2][3];
  const int a_off = (l16 * 4 + (q ^ ((l16 >> 2) & 2))) * 16;
  auto load_u = [&](int k, int n0, f32x4 (&u)[3][2]) __attribute__((always_inline)) {
    const float* bq = ub0 + (size_t)n0 * 32 + (size_t)k * 4 * CO * 32;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int h = 0; h < 2; ++h) u[nt][h] = *reinterpret_cast<const f32x4*>(bq + (size_t)nt * 16 * 32 + h * 4);
  };
  auto read_a = [&](int vstage, f32x4 (&a)[4]) __attribute__((always_inline)) {
    const char* vb = vbuf + vstage * S_V + a_off;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const f32x4*>(vb + (4 * rw + j) * (S_BT * 32));
  };

  // ---- producer state --------------------------------------------------------------------------
  const int ptid = tid - 256;
  const int plane = ptid >> 6;  // producer wave 0..3 (wave 4 + plane)
  const int pl = lane;
  int d_off[S_DPW];
  auto dma_offsets = [&](int t) __attribute__((always_inline)) {
    const Item it = item_of(t < n_items ? t : 0);
    const bool live = t < n_items;
#pragma unroll
    for (int j = 0; j < S_DPW; ++j) {
      const int s = (plane + 4 * j) * 64 + pl;
      int off = -1;
      if (live && s < S_SLOTS) {
        const int pp = s / (2 * S_PSTRIDE), rem = s - pp * (2 * S_PSTRIDE), pix = rem >> 1, half = rem & 1;
        const int py = pix / S_SIDE, px = pix - py * S_SIDE;
        const int gp = 2 * it.pair + pp;
        if (gp < n_patches && pix < S_PIX) {
          const int f = fdiv(gp, fd_frame), r = gp - f * (PY * PX);
          const int pr = fdiv(r, fd_px), pc = r - pr * PX;
          const int yy = pr * 8 - 1 + py, xx = pc * 8 - 1 + px;
          if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) off = ((f * H + yy) * W + xx) * C + half * 4;
        }
      }
      d_off[j] = off;
    }
  };
  auto issue_raw = [&](int k, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < S_DPW; ++j) {
      const void* src = d_off[j] >= 0 ? (const void*)(x + (size_t)d_off[j] + k * 8) : p.zero;
      dma16s(src, raw + stage * S_RAW + (plane + 4 * j) * 1024);
    }
  };
  // transform thread = (tile tt, channel cc), conv_wino_q's PT = 4 mapping with wid -> plane
  const int tt = ((pl >> 4) & 1) * 16 + plane * 4 + ((pl >> 3) & 1) + 2 * (pl >> 5);
  const int cc = ptid & 7;
  const int raw_off = (tt / 16) * S_PSTRIDE * 8 + (2 * ((tt / 4) % 4) * S_SIDE + 2 * (tt % 4)) * 8 + cc;
  const int v_off = (((tt & 15) * 4 + ((cc >> 1) ^ (((tt & 15) >> 2) & 2))) * 2 + (tt >> 4)) * 2 + (cc & 1);
  // transform split in two so the LDS read latency overlaps other producer work: read the 4x4 window
  // of raw(s+2) right after the barrier, compute and store V later in the interval
  auto transform_read = [&](int rstage, float (&d)[16]) __attribute__((always_inline)) {
    const float* rb = reinterpret_cast<const float*>(raw + rstage * S_RAW) + raw_off;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) d[4 * r + c] = rb[(r * S_SIDE + c) * 8];
  };
  auto transform_write = [&](const float (&d)[16], int vstage) __attribute__((always_inline)) {
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
      t[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
      t[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
      t[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
    float* vb = reinterpret_cast<float*>(vbuf + vstage * S_V) + v_off;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vb[(4 * r + 0) * S_BT * 8] = t[4 * r + 0] - t[4 * r + 2];
      vb[(4 * r + 1) * S_BT * 8] = t[4 * r + 1] + t[4 * r + 2];
      vb[(4 * r + 2) * S_BT * 8] = t[4 * r + 2] - t[4 * r + 1];
      vb[(4 * r + 3) * S_BT * 8] = t[4 * r + 1] - t[4 * r + 3];
    }
  };
  auto transform = [&](int rstage, int vstage) __attribute__((always_inline)) {
    float d[16];
    transform_read(rstage, d);
    transform_write(d, vstage);
  };
  // epilogue of item t by the producers: unit = (tile, 4 channels), conv_wino_q's arithmetic. Split in
  // two: epi_prepare (one interval ahead: output offsets, bias and residual loads in flight) and
  // epi_finish (Z rows -> output transform -> bias / residual / ReLU -> stores).
  constexpr int CQ = 12, UNITS = S_BT * CQ, UPT = (UNITS + 255) / 256;
  constexpr bool RES = EPI & 1, RELU = EPI & 2;
  const float* res = reinterpret_cast<const float*>(p.res);
  float* yout = reinterpret_cast<float*>(p.y);
  const int ps = C8 ? 8 : CO;
  const size_t oplane = (size_t)n_patches * 64 * 8;
  struct Epi {
    size_t o[UPT];
    int zo[UPT];
    bool live[UPT];
    f32x4 bias[UPT];
    f32x4 rr[UPT][RES ? 4 : 1];
  };
  // one unit per call (u: compile-time): the epilogue is spread over two intervals per side
  auto epi_prepare = [&](int t, Epi& e, int u) __attribute__((always_inline)) {
    const bool item_live = t >= 0 && t < n_items;
    const Item it = item_of(item_live ? t : 0);
    {
      const int un = ptid + 256 * u;
      const int tl = C8 ? un % S_BT : un / CQ, cq = C8 ? un / S_BT : un - tl * CQ;
      const int gp = 2 * it.pair + tl / 16;
      const bool live = item_live && un < UNITS && gp < n_patches;
      const int gpc = live ? gp : 0;
      const int f = fdiv(gpc, fd_frame), r = gpc - f * (PY * PX);
      const int pr = fdiv(r, fd_px), pc = r - pr * PX;
      const int yy = pr * 8 + 2 * ((tl / 4) % 4), xx = pc * 8 + 2 * (tl % 4);
      const int co = live ? it.n0 + 4 * cq : 0;
      const size_t pix = (size_t)(f * H + yy) * W + xx;
      e.o[u] = C8 ? (co >> 3) * oplane + pix * 8 + (co & 7) : pix * CO + co;
      e.zo[u] = tl * 48 + 4 * cq;
      e.live[u] = live;
      e.bias[u] = (p.bias && live) ? *reinterpret_cast<const f32x4*>(p.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (RES) {
#pragma unroll
        for (int px = 0; px < 4; ++px)
          e.rr[u][px] = live ? *reinterpret_cast<const f32x4*>(res + e.o[u] + (size_t)((px >> 1) * W + (px & 1)) * ps)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto epi_finish = [&](const Epi& e, int u) __attribute__((always_inline)) {
    if (e.live[u]) {
      f32x4 z[4][2];
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) {
        const f32x4* zp = reinterpret_cast<const f32x4*>(zs + i2 * S_BT * 48 + e.zo[u]);
        z[i2][0] = zp[0];
        z[i2][1] = zp[1];
      }
#pragma unroll
      for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2) {
          f32x4 v;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int h = c >> 1, ee = (c & 1) * 2 + b2;
            const float y = a2 == 0 ? z[0][h][ee] + z[1][h][ee] + z[2][h][ee] : z[1][h][ee] - z[2][h][ee] - z[3][h][ee];
            float o2 = y + e.bias[u][c];
            if constexpr (RES) o2 += e.rr[u][2 * a2 + b2][c];
            if constexpr (RELU) o2 = fmaxf(o2, 0.f);
            v[c] = o2;
          }
          *reinterpret_cast<f32x4*>(yout + e.o[u] + (size_t)(a2 * W + b2) * ps) = v;
        }
    }
  };

  // ---- the two role programs ---------------------------------------------------------------------
  // Disjoint code paths (so the consumer's accumulators are not live in the producer's code and vice
  // versa) that execute the same s_barrier sequence: 3 in the prologue, one per chunk, one to drain.
  static_assert(NCH % 2 == 0, "U / A register rotation by chunk parity");
  if (consumer) {
    const Item it0 = item_of(0);
    load_u(0, it0.n0, uu[0]);
    load_u(1, it0.n0, uu[1]);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_barrier();
    read_a(0, aa[0]);
    for (int t = 0; t < n_items; ++t) {
      const Item itc = item_of(t);
      const Item itn = item_of(t + 1 < n_items ? t + 1 : t);
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long w0 = now();
        __builtin_amdgcn_s_waitcnt(0x0070 | 6);  // U(s) landed (U(s+1) in flight); lgkmcnt(0): A(s), Z stores
        __builtin_amdgcn_s_barrier();
        stamp_wait(w0);
        __builtin_amdgcn_sched_barrier(0);  // nothing (MFMAs included) moves across an interval boundary
        const int s = t * NCH + k;  // chunk position in the block's stream
        read_a((s + 1) % 3, aa[(k + 1) & 1]);
        f32x4(&ac)[4] = aa[k & 1];
        f32x4(&uc)[3][2] = uu[k & 1];
        if (!(VAR & 32))
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
              for (int nt = 0; nt < 3; ++nt) {
                const f32x4 c0 = (k == 0 && s2 == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[j][m][nt];
                acc[j][m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][2 * m + s2], uc[nt][j >> 1][(j & 1) * 2 + s2],
                                                                     c0, 0, 0, 0);
              }
        // U(s+2) into the registers chunk s just consumed: chunk k+2 of this item or k+2-NCH of the next
        if constexpr ((VAR & 64) == 0) {
          if (k + 2 < NCH)
            load_u(k + 2, itc.n0, uu[k & 1]);
          else
            load_u(k + 2 - NCH, itn.n0, uu[k & 1]);
        }
        if (k == NCH - 1) {  // hand the item's accumulators to the producers
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int nt = 0; nt < 3; ++nt)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float m0 = acc[0][m][nt][r], m1 = acc[1][m][nt][r], m2 = acc[2][m][nt][r], m3 = acc[3][m][nt][r];
                zs[(rw * S_BT + m * 16 + 4 * q + r) * 48 + nt * 16 + l16] = f32x2{m0 + m1 + m2, m1 - m2 - m3};
              }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // Z stores
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_waitcnt(0x0070);  // past-the-end U loads
#ifdef CLASFV_KNOCKOUTS
    if constexpr ((VAR & 4) != 0) {
      if (blockIdx.x < 8 && wid == 0 && lane == 0) {
        g_wstamps[blockIdx.x][0][0] = st_wait;
        g_wstamps[blockIdx.x][0][1] = __builtin_amdgcn_s_memtime() - st_t0;
      }
    }
#endif
  } else {
    // prologue: raw(0..2) in flight, transform raw(0) and raw(1), raw(3) in flight
    dma_offsets(0);
    issue_raw(0, 0);
    issue_raw(1, 1);
    issue_raw(2, 2);
    __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * S_DPW));  // raw(0) landed
    __builtin_amdgcn_s_barrier();
    transform(0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70 | S_DPW);  // raw(1) landed
    __builtin_amdgcn_s_barrier();  // raw stage 0 read by every producer; raw(1) of every wave landed
    issue_raw(3, 0);
    transform(1, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // own V stores done
    __builtin_amdgcn_s_barrier();
    Epi ep;
#pragma unroll
    for (int u = 0; u < UPT; ++u) epi_prepare(-1, ep, u);  // no item before the first: every unit dead
    for (int t = 0; t < n_items; ++t) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        // raw(s+2) landed (raw(s+3) in flight; the previous interval's epilogue loads / stores, issued
        // before its DMAs, done too); own V stores done
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long w0 = now();
        __builtin_amdgcn_s_waitcnt(0x0070 | S_DPW);
        __builtin_amdgcn_s_barrier();
        stamp_wait(w0);
        __builtin_amdgcn_sched_barrier(0);
        const int s = t * NCH + k;
        float d[16];
        if (!(VAR & 16)) transform_read((s + 2) % 3, d);  // in flight during the epilogue below
        if (!(VAR & 8)) {
          // item t-1 (its Z rows landed before the k = 0 barrier), one unit per interval
          if (k < UPT && t > 0) epi_finish(ep, k);
          // item t: offsets, bias, residual in flight, one unit per interval
          if (k >= NCH - UPT) epi_prepare(t, ep, k - (NCH - UPT));
        }
        // raw(s+4): chunk k+4 of this item or chunk k+4-NCH of the next (offsets switch at k = NCH-4)
        if (k == NCH - 4) dma_offsets(t + 1);
        issue_raw(k + 4 < NCH ? k + 4 : k + 4 - NCH, (s + 4) % 3);
        if (!(VAR & 16)) transform_write(d, (s + 2) % 3);
      }
    }
    // drain: the last item's epilogue (its Z rows were written in the last interval)
    __builtin_amdgcn_s_waitcnt(0x0070);
    __builtin_amdgcn_s_barrier();
    if (!(VAR & 8)) {
#pragma unroll
      for (int u = 0; u < UPT; ++u) epi_finish(ep, u);
    }
    __builtin_amdgcn_s_waitcnt(0x0070);  // every DMA (past-the-end fetches included) landed before exit
#ifdef CLASFV_KNOCKOUTS
    if constexpr ((VAR & 4) != 0) {
      if (blockIdx.x < 8 && wid == 4 && lane == 0) {
        g_wstamps[blockIdx.x][1][0] = st_wait;
        g_wstamps[blockIdx.x][1][1] = __builtin_amdgcn_s_memtime() - st_t0;
      }
    }
#endif
  }
}

template <int NCH, int EPI, bool C8, int VAR = 0>
hipError_t launch_s(const ConvParams& p, hipStream_t s, int grid, int n_co, int n_patches, int n_pairs) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_wino_s<NCH, EPI, C8, VAR>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, S_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int px = p.Wo / 8, py = p.Ho / 8;
  hipLaunchKernelGGL((conv_wino_s<NCH, EPI, C8, VAR>), dim3(grid), dim3(512), S_LDS, s, p, n_co, n_patches, n_pairs,
                     fast_div(n_co), fast_div(px * py), fast_div(px));
  return hipGetLastError();
}

template <int NCH>
hipError_t launch_s_epi(const ConvParams& p, hipStream_t s, int grid, int n_co, int n_patches, int n_pairs) {
  switch ((p.res ? 1 : 0) | (p.relu ? 2 : 0)) {
    case 2:
      return p.y_c8 ? launch_s<NCH, 2, true>(p, s, grid, n_co, n_patches, n_pairs)
                    : launch_s<NCH, 2, false>(p, s, grid, n_co, n_patches, n_pairs);
    case 3: return p.y_c8 ? hipErrorInvalidValue : launch_s<NCH, 3, false>(p, s, grid, n_co, n_patches, n_pairs);
    case 1: return p.y_c8 ? hipErrorInvalidValue : launch_s<NCH, 1, false>(p, s, grid, n_co, n_patches, n_pairs);
    default: return p.y_c8 ? hipErrorInvalidValue : launch_s<NCH, 0, false>(p, s, grid, n_co, n_patches, n_pairs);
  }
}

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace

bool winos_supported(const ConvParams& p) {
  return winoq_supported(p) && p.Ho % 8 == 0 && p.Wo % 8 == 0 && (p.Cin == 64 || p.Cin == 128);
}

// p.w: conv_wino's U layout [Cin/8][4][Cout][4][4][2] (wino_transform_weights).
hipError_t launch_winos(const ConvParams& p, hipStream_t s) {
  if (!winos_supported(p)) return hipErrorInvalidValue;
  const int n_patches = p.N * p.To * (p.Ho / 8) * (p.Wo / 8);
  const int n_pairs = (n_patches + 1) / 2;
  const int n_co = p.Cout / 48;
  const int grid = n_pairs < cu_count() ? n_pairs : cu_count();
  return p.Cin == 64 ? launch_s_epi<8>(p, s, grid, n_co, n_patches, n_pairs)
                     : launch_s_epi<16>(p, s, grid, n_co, n_patches, n_pairs);
}

#ifdef CLASFV_KNOCKOUTS
// tools/convbench.hip: VAR variants of the layer1 shape (Cin 64, no residual / residual + ReLU, channels-last)
hipError_t launch_winos_var(const ConvParams& p, hipStream_t s, int var) {
  if (!winos_supported(p) || p.Cin != 64 || p.y_c8) return hipErrorInvalidValue;
  const int n_patches = p.N * p.To * (p.Ho / 8) * (p.Wo / 8);
  const int n_pairs = (n_patches + 1) / 2;
  const int n_co = p.Cout / 48;
  const int grid = n_pairs < cu_count() ? n_pairs : cu_count();
  const bool res = p.res != nullptr;
#define VARCASE(V)                                                                                  \
  case V:                                                                                           \
    return res ? launch_s<8, 3, false, V>(p, s, grid, n_co, n_patches, n_pairs)                      \
               : launch_s<8, 2, false, V>(p, s, grid, n_co, n_patches, n_pairs);
  switch (var) {
    VARCASE(0)
    VARCASE(1)
    VARCASE(2)
    VARCASE(3)
    VARCASE(4)
    VARCASE(12)
    VARCASE(20)
    VARCASE(28)
    VARCASE(36)
    VARCASE(64)
    VARCASE(68)
    VARCASE(88)
    VARCASE(92)
  }
#undef VARCASE
  return hipErrorInvalidValue;
}

void winos_stamps(unsigned long long* out) { (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wstamps), sizeof(g_wstamps)); }
#endif
