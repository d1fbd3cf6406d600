// Shared pieces of the fused Winograd F(4x4,3x3) kernels (winograd4.hip: 48 output channels per block,
// two blocks per CU; winograd4w.hip: a wide output-channel block, one block per CU): Lavin's input
// transform halves, the raw-patch ring shape and the tile-group geometry.
#pragma once
#include "common.h"

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Tile-group geometry (host-computed, wino4_geometry). Tiles are 4x4 output pixels; a flattened tile
// row is (frame, tile row) = frame * TH + ty, and a group is TR consecutive flattened rows x TC
// consecutive tile columns (segments of different frames are fine: a 1x3x3 conv never mixes frames).
struct W4Geo {
  int TR, TC;   // group shape, TR * TC <= 16 tiles
  int TH, TW;   // tiles per frame column / row
  int RP;       // 16-B LDS slots per raw patch row (a pad slot after every 4 pixels: bank spread)
  int SS;       // slots per segment (>= 6 RP: free slots shift the next segment's banks)
  int RS;       // slots per channel-half region (TR SS); region 1 = input channels 4..7
  int NI;       // DMA wave-instructions carrying data per stage (<= 4 DPW)
  int n_cob;    // output-channel blocks (cob_w channels each) per tile group
  int gpr;      // groups per flattened tile row (TW / TC)
  FastDiv fd_cob, fd_gpr, fd_th, fd_tc, fd_rp, fd_ss;
#ifdef CLASFV_KNOCKOUTS
  // conv_wino4r start stagger (convbench probe, profiles/r05ag_*: ±0): first-round block b waits
  // ((b / 8) % stagger_groups) * stagger ticks of the 100-MHz real-time clock before its first DMA
  int stagger, stagger_groups;
#endif
};

namespace {

constexpr int W4_WAVES = 4;
constexpr int W4_THREADS = 64 * W4_WAVES;
constexpr int W4_NU = 14;  // U f32x4 loads per wave per chunk (54 B operands + 2 pad)
// raw ring for DPW DMA instructions per wave per chunk (stage = 4 DPW KB): DPW = 4 (<= 16 per stage):
// 4 stages, one barrier per 2 chunks; DPW = 5, 6: 3 stages, one barrier per chunk
template <int DPW>
struct W4Ring {
  static constexpr int STAGE = W4_WAVES * DPW * 1024;
  static constexpr int NR = DPW == 4 ? 4 : 3;
  static constexpr int STEP = NR - 2;  // chunks per barrier
  static constexpr int LDS = NR * STAGE + 1024;  // + sink
};
// epilogue planes per 16 output channels: 18 column-half-0 planes [i][3] then 24 column-half-1 planes
// [i][4 (b)], each [co (stride W4_CS)][tile (16)] (a lane's 4 tiles = one 16-B store)
constexpr int W4_CS = 20;
constexpr int W4_ZS = 16 * W4_CS + 4;
constexpr int W4_ZBYTES = 42 * W4_ZS * 4;  // 54,432 B
static_assert(W4_ZBYTES <= W4Ring<4>::LDS && W4Ring<4>::LDS <= 80 * 1024 && W4Ring<5>::LDS <= 80 * 1024 &&
                  W4Ring<6>::LDS <= 80 * 1024,
              "two blocks per CU");

__device__ inline int xcd_swizzle4(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// s_waitcnt immediate waiting for vmcnt <= n (gfx9 encoding: vmcnt bits 3:0 and 15:14; expcnt and
// lgkmcnt left at their maxima)
constexpr int vm_wait(int n) { return (n & 0xF) | ((n >> 4) << 14) | 0x0F70; }


// One row half of the input transform: t[r] = (B^T d)[3 rh + r][column] from the 5 window rows
// e[q] = d[rh + q] (Lavin's B^T rows 0-2 read d rows 0-4, rows 3-5 read d rows 1-5).
template <int RH>
__device__ inline void bt_rows(const f32x2 (&e)[5], f32x2 (&t)[3]) {
  if constexpr (RH == 0) {
    t[0] = e[0] * 4.f - e[2] * 5.f + e[4];
    const f32x2 s = e[1] + e[2], u = e[3] + e[4], d = e[1] - e[2], w = e[4] - e[3];
    t[1] = u - s * 4.f;
    t[2] = w + d * 4.f;
  } else {
    const f32x2 x = e[3] - e[1], y = e[2] - e[0];
    t[0] = x + y * 2.f;
    t[1] = x - y * 2.f;
    t[2] = e[0] * 4.f - e[2] * 5.f + e[4];
  }
}

// One column half of the input transform: v[jj] = sum_c t[c] B^T[3 ch + jj][c].
template <int CH>
__device__ inline void bt_cols(const f32x2 (&t)[6], f32x2 (&v)[3]) {
  if constexpr (CH == 0) {
    v[0] = t[0] * 4.f - t[2] * 5.f + t[4];
    const f32x2 s = t[1] + t[2], u = t[3] + t[4], d = t[1] - t[2], w = t[4] - t[3];
    v[1] = u - s * 4.f;
    v[2] = w + d * 4.f;
  } else {
    const f32x2 x = t[4] - t[2], y = t[3] - t[1];
    v[0] = x + y * 2.f;
    v[1] = x - y * 2.f;
    v[2] = t[1] * 4.f - t[3] * 5.f + t[5];
  }
}

// Tile-group shape, patch pitches and DMA count for p with output-channel blocks of cob_w channels
// (false: no group of >= 12 tiles fits). Tiles
// past the map's right / bottom edge (H, W % 4 != 0) are computed on zero padding and not stored.
// fill16 (conv_wino4w): among the (TR, TC) shapes take the one with the most tiles (16 fills every MFMA
// row), then the widest; otherwise the widest TC first (the least halo per tile: conv_wino4's rule).
// At 56x56 maps (TW = 14) that is 8 rows x 2 tiles instead of 1 x 14: 16 of 16 MFMA rows carry tiles
// instead of 14, for 20 % more raw-patch bytes per tile.
inline bool wino4_geometry(const ConvParams& p, W4Geo* g, int* n_blocks, int cob_w = 48, int fill16 = 0) {
#ifdef CLASFV_KNOCKOUTS
  g->stagger = 0;
  g->stagger_groups = 1;
#endif
  if (p.Cout % cob_w || p.Cin % 8) return false;
  const int TH = (p.Ho + 3) / 4, TW = (p.Wo + 3) / 4;
  const long rows = (long)p.N * p.To * TH;  // flattened tile rows
  // TR divides one clip's tile rows (To * TH), not the batch's: the group shape -- and so whether this
  // kernel runs at all, and every clip's rounding -- depends on the per-clip shape only, never on N
  auto tr_for = [&](int tc) {
    for (int d = 16 / tc; d >= 1; --d)
      if (((long)p.To * TH) % d == 0) return d;
    return 1;
  };
  // RP, SS for a (TR, TC): fewest tiles sharing a 16-B bank quad of a 256-B row (ds_read_b64: a 32-lane
  // group = 16 tiles x one channel pair), then the 4-stage ring (<= 16 DMA instructions), then the
  // fewest DMAs; false when no pitch keeps a chunk within 24 DMA instructions
  auto pitch = [&](int TR, int TC) {
    const int PC = 4 * TC + 2, rp0 = (PC - 1) + (PC - 1) / 4 + 1;
    int best = 1 << 30;
    for (int rp = rp0; rp < rp0 + 16; ++rp)
      for (int ss = 6 * rp; ss < 6 * rp + 16; ++ss) {
        const int ni = (2 * TR * ss + 63) / 64;
        if (ni > W4_WAVES * 6) continue;
        int cnt[16] = {0}, m = 0;
        for (int t = 0; t < TR * TC; ++t) {
          const int v = ((t / TC) * ss + 5 * (t % TC)) & 15;
          if (++cnt[v] > m) m = cnt[v];
        }
        const int score = m * 1000 + (ni <= 16 ? 0 : 100) + ni;
        if (score < best) best = score, g->RP = rp, g->SS = ss;
      }
    return best != (1 << 30);
  };
  // candidates: the widest TC (conv_wino4's rule), and with fill16 the most tiles per group among
  // TC >= fill16
  int TC = 0;
  for (int d = TW < 16 ? TW : 16; d >= 1 && !TC; --d)
    if (TW % d == 0) TC = d;
  int TR = tr_for(TC);
  if (fill16) {
    int bc = TC, br = TR;
    for (int d = TW < 16 ? TW : 16; d >= fill16; --d)
      if (TW % d == 0 && tr_for(d) * d > br * bc) bc = d, br = tr_for(d);
    if ((bc != TC || br != TR) && br * bc >= 12 && pitch(br, bc)) TC = bc, TR = br;
  }
  if (TR * TC < 12 || !pitch(TR, TC)) return false;
  g->TR = TR, g->TC = TC, g->TH = TH, g->TW = TW;
  g->RS = TR * g->SS;
  g->NI = (2 * g->RS + 63) / 64;
  g->n_cob = p.Cout / cob_w;
  g->gpr = TW / TC;
  g->fd_cob = fast_div(g->n_cob);
  g->fd_gpr = fast_div(g->gpr);
  g->fd_th = fast_div(TH);
  g->fd_tc = fast_div(TC);
  g->fd_rp = fast_div(g->RP);
  g->fd_ss = fast_div(g->SS);
  *n_blocks = (int)(rows / TR) * g->gpr * g->n_cob;
  return true;
}

}  // namespace
