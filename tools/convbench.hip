// Stand-alone timing of one conv layer shape through the engine's kernels (not part of the product).
// Build + run (GPU box): bash tools/convbench.sh
//   convbench KIND N T H W CIN COUT [ITERS] [KO...]
//   KIND: wino (1x3x3 s1), winot (3x1x1 s1), sp (1x3x3 direct), tp (3x1x1 direct), pw (1x1x1),
//         spp / tpp (bf16 patch-staged 1x3x3 / 3x1x1: ko 0 conv_patch, FR*1000+S*100+NT a conv_patch
//         variant, 900 conv_dma, 901 the round-1 2-frame kernel, spatial only)
// KO = knock-out variant of the Winograd kernels (see winograd.hip): timing only, results are wrong.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd/csrc/common.h"

hipError_t launch_wino_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_winot_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_winoq_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_wino4_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_wino4w_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_winor_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_dma_x3_cfg(const ConvParams& p, int mt, int nt, int S, hipStream_t s);
hipError_t launch_dma_x3_ko(const ConvParams& p, int nt, int ko, hipStream_t s);
hipError_t launch_decoder_ko(const DecParams& p, hipStream_t s, int ko);
hipError_t launch_dma_bf16_ko(const ConvParams& p, int bn, int ko, hipStream_t s);
hipError_t launch_patch_bf16_v1(const ConvParams& p, hipStream_t s);
hipError_t launch_patch_bf16_ko(const ConvParams& p, hipStream_t s, int ko);
hipError_t launch_patch32_bf16_epi(const ConvParams& p, hipStream_t s, int epi);
hipError_t launch_patch_s2_bf16_ko(const ConvParams& p, hipStream_t s, int ko);
bool twalk_bf16_supported(const ConvParams& p);
hipError_t launch_twalk_bf16(const ConvParams& p, hipStream_t s);
hipError_t launch_twalk_bf16_ko(const ConvParams& p, hipStream_t s, int v);
hipError_t launch_twalk_x3(const ConvParams& p, hipStream_t s);
hipError_t launch_twalk_x3_ko(const ConvParams& p, hipStream_t s, int v);
void twalk_x3_weight_image(const float* w, int cout, int kp, uint16_t* out);
hipError_t launch_winoq_probe(const ConvParams& p, hipStream_t s, int ko);
void winos_stamps(unsigned long long* out);
void wino4w_stamps(unsigned long long* out, int n);
hipError_t launch_wino4r_ko(const ConvParams& p, hipStream_t s, int ko);
void wino4r_from_wino4w(const float* Uw, int cin_p, int cout_p, float* Ur);

// decoder: N clips of T x H x W, taps at (T, H/2, W/2), (T/2, H/4, W/4), (T/4, H/8), (T/8, H/16)
static int run_decoder(int N, int T, int H, int W, int iters, const std::vector<int>& kos);

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static void* dev_random(size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = lo + (hi - lo) * ((s >> 8) * (1.0f / 16777216.0f));
  }
  void* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

static void* to_bf16_dev(size_t n, float lo, float hi, unsigned seed) {
  std::vector<uint16_t> h(n);
  unsigned s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float f = lo + (hi - lo) * ((s >> 8) * (1.0f / 16777216.0f));
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
  void* d;
  CK(hipMalloc(&d, n * 2));
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: convbench KIND N T H W CIN COUT [ITERS] [KO...]\n");
    return 2;
  }
  const char* kind = argv[1];
  if (!strcmp(kind, "dec")) {
    std::vector<int> k2;
    for (int i = 7; i < argc; ++i) k2.push_back(atoi(argv[i]));
    if (k2.empty()) k2.push_back(0);
    return run_decoder(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), argc > 6 ? atoi(argv[6]) : 20, k2);
  }
  const int N = atoi(argv[2]), T = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]);
  const int Cin = atoi(argv[6]), Cout = atoi(argv[7]);
  const int iters = argc > 8 ? atoi(argv[8]) : 20;
  std::vector<int> kos;
  for (int i = 9; i < argc; ++i) kos.push_back(atoi(argv[i]));
  if (kos.empty()) kos.push_back(0);
  const bool winoqp = !strcmp(kind, "winoqp");  // conv_wino_q knock-out probes (tools/winoq_probe.hip)
  const bool winoq = !strcmp(kind, "winoq") || winoqp, winor = !strcmp(kind, "winor");
  const bool wino4 = !strcmp(kind, "wino4");  // conv_wino4 (F(4x4,3x3); no residual)
  // conv_wino4r (12 row waves): ko bits as conv_wino4r's; ko + 8192: conv_wino4w (ko - 8192) on the same
  // U values (the wino4w image, permuted for wino4r)
  const bool wino4r = !strcmp(kind, "wino4r");
  const bool wino4w = !strcmp(kind, "wino4w") || wino4r;  // conv_wino4w (wide blocks; ko: knock-outs at NTN 9)
  const bool wino = !strcmp(kind, "wino") || winoq || winor || wino4 || wino4w, winot = !strcmp(kind, "winot");
  const bool spp = !strcmp(kind, "spp"), tpp = !strcmp(kind, "tpp");  // bf16 patch-staged (conv_patch.hip)
  const bool sp = wino || spp || !strcmp(kind, "sp"), tp = winot || tpp || !strcmp(kind, "tp");
  ConvParams p;
  memset(&p, 0, sizeof(p));
  p.N = N, p.Ti = T, p.Hi = H, p.Wi = W, p.Cin = Cin;
  p.To = T, p.Ho = H, p.Wo = W, p.Cout = Cout;
  p.KT = tp ? 3 : 1, p.KH = sp ? 3 : 1, p.KW = sp ? 3 : 1;
  p.st = p.sh = p.sw = 1;
  p.pt = tp ? 1 : 0, p.ph = sp ? 1 : 0, p.pw = sp ? 1 : 0;
  // CB_STRIDE=2: the strided first conv of a block (spatial for sp, temporal for tp; direct only)
  if (getenv("CB_STRIDE") && !wino && !winot) {
    if (sp) p.sh = p.sw = 2, p.Ho = (H - 1) / 2 + 1, p.Wo = (W - 1) / 2 + 1;
    if (tp) p.st = 2, p.To = (T - 1) / 2 + 1;
  }
  // CB_BF16=1: bf16 activations/weights/outputs (direct convs only), K step 32
  const bool bf = (getenv("CB_BF16") || spp || tpp) && !wino && !winot;
  p.in_bf16 = p.out_bf16 = bf;
  p.K = p.KT * p.KH * p.KW * Cin;
  p.Kp = bf ? (p.K + 31) / 32 * 32 : (p.K + 15) / 16 * 16;
  p.M = N * p.To * p.Ho * p.Wo;
  p.relu = 1;
  if (getenv("CLASFV_NO_DMA_BUF")) p.vflags |= CLASFV_VARIANT_NO_DMA_BUF;  // conv_dma_x3's pointer-form DMAs
  if (getenv("CB_STAGGER")) p.patch_nt = atoi(getenv("CB_STAGGER"));
  if (getenv("CB_C8") && winot) p.x_c8 = 1;  // 8-channel-blocked input (the engine's mid tensors)  // conv_wino4w ko 64: sleep units per phase
  const size_t nx = (size_t)N * T * H * W * Cin, ny = (size_t)p.M * Cout;
  p.x = bf ? to_bf16_dev(nx, 0.f, 1.f, 1) : dev_random(nx, 0.f, 1.f, 1);
  const size_t nw = wino4w ? wino4w_weight_floats(Cin, Cout) : wino4 ? (size_t)(Cout / 48) * (Cin / 8) * 14336 : winor ? (size_t)24 * Cin * Cout : wino ? (size_t)16 * Cin * Cout : winot ? (size_t)6 * Cin * Cout : (size_t)Cout * p.Kp;
  p.w = bf ? to_bf16_dev(nw, -0.05f, 0.05f, 2) : dev_random(nw ? nw : 1, -0.05f, 0.05f, 2);
  p.bias = (const float*)dev_random(Cout, -0.1f, 0.1f, 3);
  p.res = (getenv("CB_NORES") || wino4 || wino4w) ? nullptr : bf ? to_bf16_dev(ny, 0.f, 1.f, 4) : dev_random(ny, 0.f, 1.f, 4);
  CK(hipMalloc(&p.y, ny * 4));
  void* w4r = nullptr;
  if (wino4r && !nw) {  // no conv_wino4w form for this Cout (NTN = 5): a random wino4r image
    w4r = dev_random(wino4r_weight_floats(Cin, Cout), -0.05f, 0.05f, 2);
  } else if (wino4r) {
    std::vector<float> uw(nw), urr(wino4r_weight_floats(Cin, Cout));
    CK(hipMemcpy(uw.data(), p.w, nw * 4, hipMemcpyDeviceToHost));
    wino4r_from_wino4w(uw.data(), Cin, Cout, urr.data());
    CK(hipMalloc(&w4r, urr.size() * 4));
    CK(hipMemcpy(w4r, urr.data(), urr.size() * 4, hipMemcpyHostToDevice));
  }
  // ko 710..719 (fp32 direct convs): conv_dma_x3 on the split-bf16 image of the same weights,
  // split-K into ko - 710 K ranges when >= 2
  void* wx3 = nullptr;
  for (int ko : kos)
    if (!wino && !winot && !bf && ((ko >= 710 && ko < 720) || (ko >= 7200 && ko < 7264)) && !wx3) {
      std::vector<float> wf(nw);
      CK(hipMemcpy(wf.data(), p.w, nw * 4, hipMemcpyDeviceToHost));
      std::vector<uint16_t> img(dma_x3_weight_elems(Cout, p.Kp));
      dma_x3_weight_image(wf.data(), Cout, p.Kp, img.data());
      CK(hipMalloc(&wx3, img.size() * 2));
      CK(hipMemcpy(wx3, img.data(), img.size() * 2, hipMemcpyHostToDevice));
    }
  // ko 1300.. (winot shapes): conv_twalk_x3 (fp32 frame walk on split-bf16 MFMAs) on its piece image of
  // random [Cout][3 Cin] weights
  void* wtx = nullptr;
  for (int ko : kos)
    if (winot && ko >= 1300 && ko < 1310 && !wtx) {
      std::vector<float> wf((size_t)Cout * 3 * Cin);
      for (size_t i = 0; i < wf.size(); ++i) wf[i] = 0.1f * (float)((i * 2654435761u) % 1000) / 1000.f - 0.05f;
      std::vector<uint16_t> img(3 * wf.size());
      twalk_x3_weight_image(wf.data(), Cout, 3 * Cin, img.data());
      CK(hipMalloc(&wtx, img.size() * 2));
      CK(hipMemcpy(wtx, img.data(), img.size() * 2, hipMemcpyHostToDevice));
    }
  for (int ko : kos)
    if (((winot && ko >= 600 && ko < 700) || (!wino && !winot && ko >= 700 && ko < 720)) && !p.part)
      CK(hipMalloc((void**)&p.part, 8 * ny * 4));  // split-K partials
  void* z;
  CK(hipMalloc(&z, 256));
  CK(hipMemset(z, 0, 256));
  p.zero = z;
  const double gflop = 2.0 * p.M * (double)Cout * Cin * p.KT * p.KH * p.KW * 1e-9;  // padded Cout
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto launch = [&](int ko) {
    if (wino4r && !(ko & 8192)) {
      ConvParams q = p;
      q.w = w4r;
      CK(ko ? launch_wino4r_ko(q, s, ko) : launch_wino4r(q, s));
    } else if (wino4w) {
      const int kw = ko & ~8192;
      CK(kw ? launch_wino4w_ko(p, s, kw) : launch_wino4w(p, s));
    }
    else if (wino4) CK(ko ? launch_wino4_ko(p, s, ko) : launch_wino4(p, s));
    else if (winor) CK(launch_winor_ko(p, s, ko));
    else if (winoqp) CK(launch_winoq_probe(p, s, ko));
    else if (winoq) CK(launch_winoq_ko(p, s, ko));
    else if (wino) CK(launch_wino_ko(p, s, ko));
    else if (winot && ko >= 1300 && ko < 1310) {  // 1300 product, 1300 + v: waves per SIMD v
      ConvParams q = p;
      q.w = wtx;
      q.Kp = 3 * Cin;
      CK(ko == 1300 ? launch_twalk_x3(q, s) : launch_twalk_x3_ko(q, s, ko - 1300));
    } else if (winot) CK(launch_winot_ko(p, s, ko));
    else if (tpp && ko == 990) CK(launch_twalk_bf16(p, s));  // conv_twalk_bf16 (frame-walking temporal conv)
    else if (tpp && ko > 990 && ko < 1200) CK(launch_twalk_bf16_ko(p, s, ko - 990));  // its PD / W forms, knock-outs
    else if (tpp && ko >= 2000 && ko < 3100) CK(launch_twalk_bf16_ko(p, s, ko - 1000));  // 128-channel forms: 1000 PD + TS
    else if ((spp || tpp) && ko == 901) CK(launch_patch_bf16_v1(p, s));
    else if (spp && ko >= 950 && ko < 970) {  // conv_patch32_bf16 (32x32x16 tiles); 951..955: NB forced;
      ConvParams q = p;                        // 960..965: direct-store epilogue
      q.patch_nt = ko % 10 ? -(ko % 10) : 0;
      CK(launch_patch32_bf16_epi(q, s, ko < 960));
    } else if (spp && ko >= 970 && ko < 1040) {  // conv_patch32_bf16 knock-outs: MODE = ko - 970
      CK(launch_patch32_bf16_epi(p, s, ko - 970));
    }
    else if ((spp || tpp) && ko != 900) CK(launch_patch_bf16_ko(p, s, ko));
    else {
      int mt, bn;
      conv_pick_tile(p.M, Cout, getenv("CB_NT") ? atoi(getenv("CB_NT")) : 0, &mt, &bn);
      if (getenv("CB_MT")) mt = atoi(getenv("CB_MT"));
      ConvParams q = p;
      if (ko >= 700 && ko < 709) q.n_split = ko - 700;  // conv_dma split-K into ko - 700 K ranges
      if (bf && ko >= 8000 && ko < 8400) {  // conv_patch_s2_bf16 (CB_STRIDE=2): ko - 8000 = S*100 + FR*10
        CK(launch_patch_s2_bf16_ko(q, s, ko - 8000));
        return;
      }
      if (bf && ko >= 7300 && ko < 7402) {  // conv_dma bf16 knock-outs (KO = ko - 7300; + 1 the pointer DMAs); 7400 / 7401: conv_dma_w, 2 / 3 stages
        CK(launch_dma_bf16_ko(q, bn, ko - 7300, s));
        return;
      }
      if (ko >= 7200 && ko < 7264) {  // conv_dma_x3 knock-outs (KO = ko - 7200; + 32 the BUF form), N tile of CB_X3CFG's NT
        q.w = wx3;
        const char* cfg = getenv("CB_X3CFG");
        int xm = 2, xn = dma_x3_bn(Cout) / 16, xs = 2;
        if (cfg && *cfg) sscanf(cfg, "%d %d %d", &xm, &xn, &xs);
        CK(launch_dma_x3_ko(q, xn, ko - 7200, s));
      } else if (ko >= 710 && ko < 720) {
        q.w = wx3;
        q.n_split = ko - 710;
        const char* cfg = getenv("CB_X3CFG");  // "MT NT S"
        int xm = 2, xn = dma_x3_bn(Cout) / 16, xs = 2;
        if (cfg && *cfg) sscanf(cfg, "%d %d %d", &xm, &xn, &xs);
        CK(launch_dma_x3_cfg(q, xm, xn, xs, s));
      } else {
        CK(launch_conv(q, mt, bn, s));
      }
    }
  };
  // warm every variant up (clocks settle), then interleave 3 timed rounds and keep each one's best
  for (int ko : kos)
    for (int i = 0; i < 10; ++i) launch(ko);
  std::vector<float> best(kos.size(), 1e30f);
  for (int rep = 0; rep < 3; ++rep)
    for (size_t v = 0; v < kos.size(); ++v) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < iters; ++i) launch(kos[v]);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= iters;
      if (ms < best[v]) best[v] = ms;
    }
  if (winoq)
    for (int ko : kos)
      if (ko == 12 || ko == 20 || ko == 28 || ko == 36 || ko == 44 || ko == 76 || ko == 100) {  // conv_wino_s stamps: per block, consumer / producer wait + barrier vs total cycles
        CK(hipDeviceSynchronize());
        launch(ko);  // the stamps of this variant
        CK(hipDeviceSynchronize());
        unsigned long long st[8][2][2];
        winos_stamps(&st[0][0][0]);
        printf("ko %d\n", ko);
        for (int bl = 0; bl < 8; ++bl)
          printf("stamps block %d: consumer wait %llu / %llu (%.3f), producer wait %llu / %llu (%.3f)\n", bl,
                 st[bl][0][0], st[bl][0][1], st[bl][0][1] ? (double)st[bl][0][0] / st[bl][0][1] : 0.0, st[bl][1][0],
                 st[bl][1][1], st[bl][1][1] ? (double)st[bl][1][0] / st[bl][1][1] : 0.0);
      }
  if (wino4w)
    for (int ko : kos)
      if ((ko & ~8192) == 512) {  // conv_wino4w / conv_wino4r per-block stamps (s_memrealtime, 100 MHz)
        const bool two = false;
        CK(hipDeviceSynchronize());
        launch(ko);
        CK(hipDeviceSynchronize());
        const int n = 16384;
        std::vector<unsigned long long> st((size_t)n * 10);
        wino4w_stamps(st.data(), n);
        auto S = [&](int b, int i) { return st[(size_t)b * 10 + i]; };
        const int last = two ? 6 : 3;
        int nb = 0;
        while (nb < n && S(nb, last) != 0) ++nb;
        double ph[6] = {0, 0, 0, 0, 0, 0}, tot = 0;
        unsigned long long t_min = ~0ull, t_max = 0;
        for (int b = 0; b < nb; ++b) {
          for (int i = 0; i < last; ++i) ph[i] += (double)S(b, i + 1) - (double)S(b, i);
          tot += S(b, last) - S(b, 0);
          t_min = S(b, 0) < t_min ? S(b, 0) : t_min;
          t_max = S(b, last) > t_max ? S(b, last) : t_max;
        }
        std::vector<int> idx(nb);
        for (int b = 0; b < nb; ++b) idx[b] = b;
        auto key = [&](int b) { return (S(b, 9) & 0xf) * 65536 + ((S(b, 8) >> 8) & 0xff); };
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return key(a) != key(b) ? key(a) < key(b) : S(a, 0) < S(b, 0); });
        double gap = 0;
        int ng = 0, ncu = 0;
        for (int i = 0; i < nb; ++i) {
          if (i == 0 || key(idx[i]) != key(idx[i - 1])) {
            ++ncu;
            continue;
          }
          gap += (double)S(idx[i], 0) - (double)S(idx[i - 1], last);
          ++ng;
        }
        printf("stamps ko %d: %d blocks on %d CUs, wall %.1f us; per block (us):", ko, nb, ncu, (t_max - t_min) / 100.0);
        const char* names[6] = {"prologue", "chunk loop", "epilogue", "item-2 prologue", "item-2 chunk loop", "item-2 epilogue"};
        for (int i = 0; i < last; ++i) printf(" %s %.2f,", names[i], ph[i] / nb / 100.0);
        printf(" total %.2f; CU gap between blocks %.2f us\n", tot / nb / 100.0, ng ? gap / ng / 100.0 : 0.0);
        // phase alignment across CUs: blocks in their epilogue (stamp 2 .. 3) at each 0.5-us sample of the
        // middle 80 % of the run -- lockstep blocks give a bursty count (all CUs writing at once),
        // de-phased ones a flat count near ncu x epilogue / block time
        if (!two && nb > 0) {
          const unsigned long long a0 = t_min + (t_max - t_min) / 10, a1 = t_max - (t_max - t_min) / 10;
          std::vector<int> cnt((size_t)((a1 - a0) / 50 + 1), 0);
          for (int b = 0; b < nb; ++b)
            for (unsigned long long t = S(b, 2); t < S(b, 3); t += 1)
              if (t >= a0 && t < a1 && (t - a0) % 50 == 0) ++cnt[(t - a0) / 50];
          std::vector<int> sc = cnt;
          std::sort(sc.begin(), sc.end());
          double mean = 0;
          for (int c : sc) mean += c;
          mean /= sc.size();
          printf("epilogue concurrency (blocks per 0.5-us sample): mean %.1f, p10 %d, p50 %d, p90 %d, max %d (flat: %.1f)\n", mean,
                 sc[sc.size() / 10], sc[sc.size() / 2], sc[sc.size() * 9 / 10], sc.back(), ncu * ph[2] / tot);
        }
      }
  for (size_t v = 0; v < kos.size(); ++v)
    printf("%s%s%-6s N=%d T=%d H=%d W=%d Cin=%d Cout=%d ko=%-3d  %8.3f ms  %7.1f TF(alg)\n", p.res ? "res   " : "nores ", bf ? "bf16 " : "",
           kind, N, T, H, W, Cin, Cout, kos[v], best[v], gflop / best[v]);
  // CB_CHECK=1: every variant's output against the first one's (bitwise; max |diff| printed)
  if (getenv("CB_CHECK") && kos.size() > 1) {
    std::vector<float> ref(ny), got(ny);
    auto fetch = [&](std::vector<float>& out) {  // bf16 outputs widened to float
      if (!bf) {
        CK(hipMemcpy(out.data(), p.y, ny * 4, hipMemcpyDeviceToHost));
        return;
      }
      std::vector<uint16_t> h(ny);
      CK(hipMemcpy(h.data(), p.y, ny * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < ny; ++i) {
        const uint32_t u = (uint32_t)h[i] << 16;
        memcpy(&out[i], &u, 4);
      }
    };
    CK(hipMemset(p.y, 0, ny * 4));
    launch(kos[0]);
    CK(hipDeviceSynchronize());
    fetch(ref);
    for (size_t v = 1; v < kos.size(); ++v) {
      CK(hipMemset(p.y, 0, ny * 4));
      launch(kos[v]);
      CK(hipDeviceSynchronize());
      fetch(got);
      size_t nd = 0;
      double md = 0;
      for (size_t i = 0; i < ny; ++i)
        if (got[i] != ref[i]) {
          ++nd;
          const double d = fabs((double)got[i] - (double)ref[i]);
          if (d > md || d != d) md = d;
        }
      printf("check ko=%d vs ko=%d: %zu of %zu differ, max |diff| %.3e%s\n", kos[v], kos[0], nd, ny, md,
             nd ? "" : " (bit-identical)");
    }
  }
  return 0;
}

static float scale_ac(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

static int run_decoder(int N, int T, int H, int W, int iters, const std::vector<int>& kos) {
  DecParams d;
  memset(&d, 0, sizeof(d));
  const int div[4][2] = {{1, 2}, {2, 4}, {4, 8}, {8, 16}};
  for (int i = 0; i < 4; ++i) {
    DecTap& t = d.tap[i];
    t.T = T / div[i][0];
    t.H = H / div[i][1];
    t.W = W / div[i][1];
    t.st = scale_ac(t.T, T);
    t.sh = scale_ac(t.H, H);
    t.sw = scale_ac(t.W, W);
    t.p = (const float*)dev_random((size_t)N * t.T * t.H * t.W * 64, -1.f, 1.f, 10 + i);
  }
  d.b1 = (const float*)dev_random(64, -0.1f, 0.1f, 20);
  d.w2 = (const float*)dev_random(64 * 64, -0.1f, 0.1f, 21);
  d.b2 = (const float*)dev_random(64, -0.1f, 0.1f, 22);
  d.wh = (const float*)dev_random(8 * 64, -0.1f, 0.1f, 23);
  d.bh = (const float*)dev_random(8, -0.1f, 0.1f, 24);
  CK(hipMalloc((void**)&d.seg, (size_t)N * 2 * T * H * W * 4));
  CK(hipMalloc((void**)&d.mot, (size_t)N * 4 * T * H * W * 4));
  d.N = N, d.T = T, d.H = H, d.W = W;
  CK(hipMalloc(&d.idx, decoder_index_bytes(T, H, W)));
  d.bf16 = getenv("CB_BF16") ? 1 : 0;
  if (getenv("CB_X3") || d.bf16) {  // split-bf16 comb_2 (X3) and heads: W2 / Wh pieces in lane order
    std::vector<float> w2(64 * 64), wh(8 * 64);
    CK(hipMemcpy(w2.data(), d.w2, w2.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(wh.data(), d.wh, wh.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint16_t> xb(DECODER_X3_ELEMS);
    decoder_x3_weights(w2.data(), wh.data(), xb.data());
    void* dx;
    CK(hipMalloc(&dx, xb.size() * 2));
    CK(hipMemcpy(dx, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
    d.w2x3 = dx;
    d.x3 = getenv("CB_X3") ? 1 : 0;
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // outputs of every variant against the first one's (seg logits and tanh(motion))
  const size_t nseg = (size_t)N * 2 * T * H * W, nmot = (size_t)N * 4 * T * H * W;
  std::vector<float> ref(nseg + nmot), got(nseg + nmot);
  for (size_t v = 0; v < kos.size(); ++v) {
    CK(hipMemset(d.seg, 0, nseg * 4));
    CK(hipMemset(d.mot, 0, nmot * 4));
    CK(launch_decoder_ko(d, s, kos[v]));
    CK(hipStreamSynchronize(s));
    std::vector<float>& o = v ? got : ref;
    CK(hipMemcpy(o.data(), d.seg, nseg * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o.data() + nseg, d.mot, nmot * 4, hipMemcpyDeviceToHost));
    if (!v) continue;
    size_t nd = 0;
    double md = 0;
    for (size_t i = 0; i < o.size(); ++i)
      if (memcmp(&ref[i], &got[i], 4)) {
        ++nd;
        md = fmax(md, fabs((double)ref[i] - got[i]));
      }
    printf("check dec ko=%d vs ko=%d: %zu of %zu differ, max |diff| %.3e\n", kos[v], kos[0], nd, o.size(), md);
  }
  for (int ko : kos)
    for (int i = 0; i < 5; ++i) CK(launch_decoder_ko(d, s, ko));
  std::vector<float> best(kos.size(), 1e30f);
  for (int rep = 0; rep < 3; ++rep)
    for (size_t v = 0; v < kos.size(); ++v) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < iters; ++i) CK(launch_decoder_ko(d, s, kos[v]));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms / iters < best[v]) best[v] = ms / iters;
    }
  for (size_t v = 0; v < kos.size(); ++v)
    printf("dec    N=%d T=%d H=%d W=%d ko=%-3d  %8.3f ms\n", N, T, H, W, kos[v], best[v]);
  return 0;
}
