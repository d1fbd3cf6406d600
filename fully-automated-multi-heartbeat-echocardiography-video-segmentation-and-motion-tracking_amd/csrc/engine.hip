// CLAS-FV engine: network plan, weight folding, workspace arena and the C ABI (include/clasfv.h).
//
// Reference module: R2plus1D_18_MotionNet (src/model/R2plus1D_18_MotionNet.py:10-71) on top of
// torchvision 0.6.0 r2plus1d_18. The 242 state-dict entries are accepted under the reference key
// names (optionally "module."-prefixed, motion_segment.py:69-72); clasfv_finalize folds every
// eval-mode BatchNorm into the preceding convolution, pads channel counts for the kernels
// (45->48, 230->240, 460->480, 921->960) and uploads everything to HBM once.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "clasfv.h"
#include "common.h"
#include "plumbing.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(CLASFV_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

constexpr double kBnEps = 1e-5;

struct Param {
  std::string name;
  std::vector<int64_t> shape;
  std::vector<float> data;
  bool loaded = false;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    return n;
  }
};

int round_up(int x, int m) { return (x + m - 1) / m * m; }

// Padded channel count of an activation tensor: a multiple of the K step (16 fp32 / 32 bf16
// channels) whose 16-channel count has a divisor in {9,8,6,5,4,3} (a legal N tile). The network
// input keeps 3 + 1 fp32 channels (stem kernel).
int pad_channels(int c, bool bf16) {
  if (c == 3) return 4;
  const int step = bf16 ? 32 : 16;
  int cp = round_up(c, step);
  auto ok = [](int cp_) {
    for (int nt : {9, 8, 6, 5, 4, 3})
      if ((cp_ / 16) % nt == 0) return true;
    return false;
  };
  while (!ok(cp)) cp += step;
  return cp;
}

enum Role { STEM_S, STEM_T, SP1, TP1, SP2, TP2, DS, PROJ };

struct Conv {
  Role role;
  std::string w, bn;  // parameter name prefixes (".weight" / BN module)
  int cin, cout, cin_p, cout_p;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int K, Kp, cout_alloc;
  int cin2 = 0;  // second input of a dual 1x1x1 conv (decoder P01 = W0 f_stem + W1 f_layer1)
  int stem = 0, in_bf16 = 0, out_bf16 = 0;
  void* dw = nullptr;     // weights, dtype of the conv's input
  float* db = nullptr;    // folded-BN bias (fp32)
  float* dwino = nullptr;  // Winograd F(2x2,3x3) transformed weights (fp32 stride-1 1x3x3 convs)
  float* dwino4 = nullptr;  // Winograd F(4x4,3x3) transformed weights (the same convs, cout_p % 48 == 0)
  float* dwino4w = nullptr;  // the same for conv_wino4w's wide output-channel blocks (wino4w_ntn(cout_p) > 0)
  float* dwino4r = nullptr;  // the same values in conv_wino4r's (12 row waves) order
  float* dwinot = nullptr;  // Winograd F(4,3)-in-time transformed weights (fp32 stride-1 3x1x1 convs)
  void* dws16 = nullptr;    // bf16 stem weights, hi and lo images [64][7 kh][8 kw][4 c] (bf16 engines);
                            // fp32 engines: hi, mid and lo images [48][7][8][4] (conv_stem_x3)
  void* dx3 = nullptr;      // fp32 engines' implicit-GEMM convs: 3-piece bf16 image for conv_dma_x3
};

// fp32 stride-1 3x1x1 convs run on the fused temporal Winograd kernel, fp32 stride-1 1x3x3 convs on
// the fused spatial one (CLASFV_VARIANT_NO_WINOGRAD: both on the direct implicit GEMM).
bool use_winot(const Conv& c, bool bf16, int vflags) {
  if (vflags & CLASFV_VARIANT_NO_WINOGRAD) return false;
  return !bf16 && (c.role == STEM_T || c.role == TP1 || c.role == TP2) && c.kt == 3 && c.kh == 1 && c.kw == 1 &&
         c.st == 1 && c.cin_p % 8 == 0 && c.cout_p % 64 == 0;
}

bool use_wino(const Conv& c, bool bf16, int vflags) {
  if (vflags & CLASFV_VARIANT_NO_WINOGRAD) return false;
  return !bf16 && (c.role == SP1 || c.role == SP2) && c.kt == 1 && c.kh == 3 && c.kw == 3 && c.sh == 1 &&
         c.sw == 1 && c.cin_p % 16 == 0 && c.cout_p % 48 == 0;
}

// Kernel-variant flags and tuning overrides from the environment (read once, at clasfv_create).
int env_variants() {
  auto on = [](const char* n) { return getenv(n) != nullptr; };
  const char* w = getenv("CLASFV_WINOGRAD");
  const char* ts1 = getenv("CLASFV_WINOT_TS1");
  int f = 0;
  if (w && w[0] == '0') f |= CLASFV_VARIANT_NO_WINOGRAD;
  if (on("CLASFV_NO_WINO_PATCH")) f |= CLASFV_VARIANT_NO_WINO_PATCH;
  if (on("CLASFV_WINOT_REFERENCE")) f |= CLASFV_VARIANT_WINOT_REFERENCE;
  if (on("CLASFV_NO_C8")) f |= CLASFV_VARIANT_NO_C8;
  if (on("CLASFV_NO_STEM_BF16")) f |= CLASFV_VARIANT_NO_STEM_BF16;
  if (on("CLASFV_NO_PATCH_BF16")) f |= CLASFV_VARIANT_NO_PATCH_BF16;
  if (on("CLASFV_NO_DECODER_BF16")) f |= CLASFV_VARIANT_NO_DECODER_BF16;
  if (ts1 && ts1[0] == '0') f |= CLASFV_VARIANT_WINOT_NO_TS1;
  if (on("CLASFV_NO_SPLIT_K")) f |= CLASFV_VARIANT_NO_SPLIT_K;
  if (on("CLASFV_NO_WINO4")) f |= CLASFV_VARIANT_NO_WINO4;
  if (on("CLASFV_NO_DECODER_X3")) f |= CLASFV_VARIANT_NO_DECODER_X3;
  if (on("CLASFV_NO_DMA_X3")) f |= CLASFV_VARIANT_NO_DMA_X3;
  if (on("CLASFV_NO_STEM_X3")) f |= CLASFV_VARIANT_NO_STEM_X3;
  if (on("CLASFV_NO_WINO4W")) f |= CLASFV_VARIANT_NO_WINO4W;
  if (on("CLASFV_NO_PATCH32")) f |= CLASFV_VARIANT_NO_PATCH32;
  if (on("CLASFV_NO_PROJ_X3")) f |= CLASFV_VARIANT_NO_PROJ_X3;
  if (on("CLASFV_NO_WINO4R")) f |= CLASFV_VARIANT_NO_WINO4R;
  if (on("CLASFV_NO_DMA_BUF")) f |= CLASFV_VARIANT_NO_DMA_BUF;
  if (on("CLASFV_W4R_CACHED_STORES")) f |= CLASFV_VARIANT_W4R_CACHED_STORES;
  if (on("CLASFV_PATCH32_CACHED_STORES")) f |= CLASFV_VARIANT_PATCH32_CACHED_STORES;
  if (on("CLASFV_NO_DMA_W")) f |= CLASFV_VARIANT_NO_DMA_W;
  if (on("CLASFV_NO_TWALK")) f |= CLASFV_VARIANT_NO_TWALK;
  return f;
}

// every CLASFV_VARIANT_* bit of include/clasfv.h (the retired bits are rejected)
constexpr int kVariantMask = CLASFV_VARIANT_NO_WINOGRAD | CLASFV_VARIANT_NO_WINO_PATCH | CLASFV_VARIANT_WINOT_REFERENCE |
                             CLASFV_VARIANT_NO_C8 | CLASFV_VARIANT_NO_STEM_BF16 | CLASFV_VARIANT_NO_PATCH_BF16 |
                             CLASFV_VARIANT_NO_DECODER_BF16 | CLASFV_VARIANT_WINOT_NO_TS1 | CLASFV_VARIANT_NO_SPLIT_K |
                             CLASFV_VARIANT_NO_WINO4 | CLASFV_VARIANT_NO_DECODER_X3 | CLASFV_VARIANT_NO_DMA_X3 |
                             CLASFV_VARIANT_NO_STEM_X3 | CLASFV_VARIANT_NO_WINO4W | CLASFV_VARIANT_NO_PATCH32 |
                             CLASFV_VARIANT_NO_PROJ_X3 | CLASFV_VARIANT_NO_WINO4R | CLASFV_VARIANT_NO_DMA_BUF |
                             CLASFV_VARIANT_W4R_CACHED_STORES | CLASFV_VARIANT_PATCH32_CACHED_STORES |
                             CLASFV_VARIANT_NO_DMA_W | CLASFV_VARIANT_NO_TWALK;

int env_int(const char* name) {
  const char* e = getenv(name);
  return e ? atoi(e) : 0;
}

// Channel padding, K extent and dtypes of one conv for the engine's compute dtype.
void layout_conv(Conv& c, bool bf16) {
  c.stem = (c.role == STEM_S);
  c.in_bf16 = bf16 && !c.stem;
  c.out_bf16 = bf16 && c.role != PROJ;
  c.cin_p = pad_channels(c.cin, bf16);
  c.cout_p = c.role == PROJ ? c.cout : pad_channels(c.cout, bf16);
  c.K = c.kt * c.kh * c.kw * c.cin_p + c.cin2;
  c.Kp = round_up(c.K, c.in_bf16 ? 32 : 16);
  c.cout_alloc = c.cout_p;  // every tile width used divides cout_p
}

Conv make_conv(Role role, const std::string& w, const std::string& bn, int cin, int cout, int kt, int kh, int kw,
               int st, int sh, int sw, int pt, int ph, int pw) {
  Conv c;
  c.role = role;
  c.w = w;
  c.bn = bn;
  c.cin = cin;
  c.cout = cout;
  c.kt = kt, c.kh = kh, c.kw = kw, c.st = st, c.sh = sh, c.sw = sw, c.pt = pt, c.ph = ph, c.pw = pw;
  layout_conv(c, false);
  return c;
}

int midplanes(int i, int o) { return (i * o * 27) / (i * 9 + 3 * o); }

// Engine-wide kernel switches: CLASFV_VARIANT_* flags and the implicit-GEMM / patch-kernel tile
// overrides (0: automatic).
struct Tuning {
  int vflags = 0, conv_nt = 0, patch_nt = 0;
};

}  // namespace

struct clasfv_engine {
  int device = 0;
  std::vector<Param> params;
  std::unordered_map<std::string, int> index;
  std::vector<Conv> convs;  // backbone, execution order
  Conv proj[5];             // decoder projections (stem, layer1..4) -> 64 channels
  float *b1 = nullptr, *w2 = nullptr, *b2 = nullptr, *wh = nullptr, *bh = nullptr;
  void* w2x3 = nullptr;  // W2 as three bf16 pieces in the decoder's MFMA lane order (fp32 engines)
  bool ready = false;
  int dtype = CLASFV_DTYPE_FP32;  // compute dtype of the encoder convs
  Tuning tune;                    // kernel variants / tile overrides (environment at create)
  float* zero = nullptr;  // 256 zero bytes for padding taps
  // One forward context per launch stream: the workspace arena (activations, mid tensors, decoder taps
  // and index table) and the side stream with its fork / join events. The decoder projections of the
  // stem/layer1, layer2 and layer3 taps run on the side stream as soon as their tap exists, filling the
  // CUs the backbone's later (small-grid) convs leave idle; the decoder waits for them (events, no host
  // synchronisation). Forwards issued on different streams own different contexts, so they may run
  // concurrently on one handle (a serving pipeline with two videos in flight): each one's arena is
  // touched only by work ordered on its own stream. Forwards on one stream reuse its context in order.
  struct Ctx {
    hipStream_t stream = nullptr;  // the launch stream this context belongs to
    char* arena = nullptr;
    size_t arena_bytes = 0;
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint64_t last_use = 0;
  };
  std::vector<Ctx*> ctxs;
  uint64_t ctx_clock = 0;
  // per-kernel HIP-event timing of clasfv_forward (clasfv_set_kernel_timing)
  bool ktime = false;
  std::vector<hipEvent_t> evs;  // event pool; evs[0..nev) recorded since the last read
  int nev = 0;
  struct Rec {
    const char* name;
    double gflop;   // algorithmic (direct-convolution MACs x 2, unpadded channels)
    double xgflop;  // MFMA work the launch executes (Winograd-domain products, padded channels/tiles)
    int e0, e1;
  };
  std::vector<Rec> recs;
};

namespace {

void add_param(clasfv_engine* e, const std::string& name, std::vector<int64_t> shape) {
  Param p;
  p.name = name;
  p.shape = std::move(shape);
  e->index[name] = (int)e->params.size();
  e->params.push_back(std::move(p));
}

void add_bn(clasfv_engine* e, const std::string& pre, int c) {
  add_param(e, pre + ".weight", {c});
  add_param(e, pre + ".bias", {c});
  add_param(e, pre + ".running_mean", {c});
  add_param(e, pre + ".running_var", {c});
  add_param(e, pre + ".num_batches_tracked", {});
}

// Build the layer plan and the state-dict table in the reference's registration order.
void build_plan(clasfv_engine* e) {
  const std::string R = "r2plus1d_model.";
  auto reg = [&](const Conv& c) {
    add_param(e, c.w + ".weight", {c.cout, c.cin, c.kt, c.kh, c.kw});
    add_bn(e, c.bn, c.cout);
    e->convs.push_back(c);
  };
  reg(make_conv(STEM_S, R + "stem.0", R + "stem.1", 3, 45, 1, 7, 7, 1, 2, 2, 0, 3, 3));
  reg(make_conv(STEM_T, R + "stem.3", R + "stem.4", 45, 64, 3, 1, 1, 1, 1, 1, 1, 0, 0));
  int inplanes = 64;
  const int planes_l[4] = {64, 128, 256, 512}, stride_l[4] = {1, 2, 2, 2};
  for (int li = 0; li < 4; ++li) {
    const int planes = planes_l[li], stride = stride_l[li];
    for (int b = 0; b < 2; ++b) {
      const int st = b == 0 ? stride : 1;
      const int cin1 = b == 0 ? inplanes : planes;
      const int mid = midplanes(cin1, planes);
      const std::string pre = R + "layer" + std::to_string(li + 1) + "." + std::to_string(b) + ".";
      reg(make_conv(SP1, pre + "conv1.0.0", pre + "conv1.0.1", cin1, mid, 1, 3, 3, 1, st, st, 0, 1, 1));
      reg(make_conv(TP1, pre + "conv1.0.3", pre + "conv1.1", mid, planes, 3, 1, 1, st, 1, 1, 1, 0, 0));
      reg(make_conv(SP2, pre + "conv2.0.0", pre + "conv2.0.1", planes, mid, 1, 3, 3, 1, 1, 1, 0, 1, 1));
      reg(make_conv(TP2, pre + "conv2.0.3", pre + "conv2.1", mid, planes, 3, 1, 1, 1, 1, 1, 1, 0, 0));
      if (b == 0 && (stride != 1 || inplanes != planes))
        reg(make_conv(DS, pre + "downsample.0", pre + "downsample.1", inplanes, planes, 1, 1, 1, stride, stride,
                      stride, 0, 0, 0));
    }
    inplanes = planes;
  }
  add_param(e, R + "fc.weight", {400, 512});
  add_param(e, R + "fc.bias", {400});
  add_param(e, "comb_1_layer.weight", {64, 1024, 1, 1, 1});
  add_param(e, "comb_1_layer.bias", {64});
  add_bn(e, "comb_batch_norm_1", 64);
  add_param(e, "comb_2_layer.weight", {64, 64, 1, 1, 1});
  add_param(e, "comb_2_layer.bias", {64});
  add_bn(e, "comb_batch_norm_2", 64);
  add_param(e, "motion_head.weight", {4, 64, 1, 1, 1});
  add_param(e, "motion_head.bias", {4});
  add_param(e, "segmentation_head.weight", {2, 64, 1, 1, 1});
  add_param(e, "segmentation_head.bias", {2});
  // decoder projections: proj[0] is the dual 1x1x1 conv over (stem, layer1) -> P01; proj[1] unused
  const int tap_c[5] = {64, 64, 128, 256, 512};
  for (int i = 0; i < 5; ++i) e->proj[i] = make_conv(PROJ, "", "", tap_c[i], 64, 1, 1, 1, 1, 1, 1, 0, 0, 0);
  e->proj[0].cin2 = 64;
  layout_conv(e->proj[0], false);
}

const std::vector<float>& P(clasfv_engine* e, const std::string& n) { return e->params[e->index.at(n)].data; }

void bn_scale_shift(clasfv_engine* e, const std::string& bn, int c, std::vector<double>& s, std::vector<double>& t) {
  const auto& g = P(e, bn + ".weight");
  const auto& b = P(e, bn + ".bias");
  const auto& m = P(e, bn + ".running_mean");
  const auto& v = P(e, bn + ".running_var");
  s.resize(c);
  t.resize(c);
  for (int i = 0; i < c; ++i) {
    s[i] = (double)g[i] / sqrt((double)v[i] + kBnEps);
    t[i] = (double)b[i] - (double)m[i] * s[i];
  }
}

int upload(const std::vector<float>& h, float** d) {
  HIP_TRY(hipMalloc(d, h.size() * sizeof(float)));
  HIP_TRY(hipMemcpy(*d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  return CLASFV_OK;
}

// float -> bf16 bits, round to nearest even (weights are finite).
uint16_t to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

int upload_bf16(const std::vector<float>& h, void** d) {
  std::vector<uint16_t> b(h.size());
  for (size_t i = 0; i < h.size(); ++i) b[i] = to_bf16(h[i]);
  HIP_TRY(hipMalloc(d, b.size() * sizeof(uint16_t)));
  HIP_TRY(hipMemcpy(*d, b.data(), b.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  return CLASFV_OK;
}

// Folded, padded [cout_alloc][Kp] weight image of one conv. `wsrc(o, c, tap)` returns the raw weight.
template <class F>
int upload_conv(Conv& c, F wsrc, const std::vector<double>& scale, const std::vector<double>& shift, bool has_bias) {
  std::vector<float> w((size_t)c.cout_alloc * c.Kp, 0.f);
  const int taps = c.kt * c.kh * c.kw;
  for (int o = 0; o < c.cout; ++o)
    for (int tap = 0; tap < taps; ++tap)
      for (int ci = 0; ci < c.cin; ++ci)
        w[(size_t)o * c.Kp + (size_t)tap * c.cin_p + ci] = (float)((double)wsrc(o, ci, tap) * scale[o]);
  int rc = c.in_bf16 ? upload_bf16(w, &c.dw) : upload(w, reinterpret_cast<float**>(&c.dw));
  if (rc) return rc;
  if (!c.in_bf16 && !c.stem && c.Kp % 16 == 0) {  // conv_dma_x3's split image of the same weights
    std::vector<uint16_t> x3(dma_x3_weight_elems(c.cout_alloc, c.Kp));
    dma_x3_weight_image(w.data(), c.cout_alloc, c.Kp, x3.data());
    HIP_TRY(hipMalloc(&c.dx3, x3.size() * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(c.dx3, x3.data(), x3.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  }
  if (has_bias) {
    std::vector<float> b(c.cout_alloc, 0.f);
    for (int o = 0; o < c.cout; ++o) b[o] = (float)shift[o];
    rc = upload(b, &c.db);
  }
  return rc;
}

struct Shape5 {
  int n, t, h, w, c;
  size_t numel() const { return (size_t)n * t * h * w * c; }
};

// Algorithmic FLOPs of one conv (2 per MAC over the unpadded channels).
double conv_gflop(const Conv& c, const Shape5& out) {
  const double m = (double)out.n * out.t * out.h * out.w;
  return 2.0 * m * c.cout * (double)(c.cin + c.cin2) * c.kt * c.kh * c.kw * 1e-9;
}

// MFMA work one launch of kernel `kname` executes for conv c (2 FLOP per multiply-add issued to
// the matrix cores, padded channels and partial tiles included): Winograd F(2x2,3x3) issues 16
// products per 2x2 output tile and (input, output) channel pair instead of 36, F(2x4,3x3) 24 per
// 2x4 tile instead of 72, F(4,3) in time 6 per 4 frames instead of 12; the implicit GEMMs issue
// ceil(M / BM) * BM rows x cout_p x Kp.
double conv_exec_gflop(const Conv& c, const Shape5& out, const char* kname) {
  const double nt = (double)out.n * out.t;
  const double cc = (double)c.cin_p * c.cout_p;
  if (!strcmp(kname, "conv_wino4") || !strcmp(kname, "conv_wino4w") || !strcmp(kname, "conv_wino4r")) {  // F(4x4,3x3): 36 products per 4x4
    ConvParams p{};                                                           // tile and channel pair, 16-tile groups
    p.N = out.n, p.Ti = p.To = out.t, p.Hi = p.Ho = out.h, p.Wi = p.Wo = out.w;
    p.Cin = c.cin_p, p.Cout = c.cout_p;
    return kname[10] == 'r' ? wino4r_exec_gflop(p) : kname[10] == 'w' ? wino4w_exec_gflop(p) : wino4_exec_gflop(p);
  }
  if (!strcmp(kname, "conv_wino_q") || !strcmp(kname, "conv_wino"))
    return 2.0 * nt * ((out.h + 1) / 2) * ((out.w + 1) / 2) * 16.0 * cc * 1e-9;
  if (!strcmp(kname, "conv_winot")) return 2.0 * out.n * (out.t / 4) * (double)out.h * out.w * 6.0 * cc * 1e-9;
  // Split-bf16 ("x3") kernels of the fp32 engines run on the bf16 matrix pipe: their work is counted
  // in that pipe's own products, six bf16 products per product of the fp32 GEMM they compute (the
  // f32-MFMA kernels count f32 products), so each kernel's rate compares with the peak of the pipe it
  // issues to (bench.py rates them against 2.5 PFLOP/s, the f32 ones against 157.3 TFLOP/s).
  if (!strcmp(kname, "conv_stem_x3"))  // 6 x the fp32 GEMM (K = 7 rows x 8 taps x 4 channels)
    return 6 * 2.0 * ceil((double)out.n * out.t * out.h * out.w / 256.0) * 256.0 * 48.0 * 224.0 * 1e-9;
  if (!strcmp(kname, "conv_stem_bf16"))
    return 3 * 2.0 * ceil((double)out.n * out.t * out.h * out.w / 256.0) * 256.0 * 64.0 * 224.0 * 1e-9;
  if (!strcmp(kname, "conv_patch_bf16")) {  // frames x 64-pixel tiles: 2 x 8x8 for 1x3x3, 4 x 64 flat for 3x1x1
    const int fr = c.kt == 1 ? 2 : 4;
    const double px = c.kt == 1 ? (double)((out.h + 7) / 8 * 8) * ((out.w + 7) / 8 * 8)
                                : (double)((out.h * out.w + 63) / 64 * 64);
    return 2.0 * out.n * ((out.t + fr - 1) / fr * fr) * px * c.cout_p * (double)c.Kp * 1e-9;
  }
  if (!strcmp(kname, "conv_proj_x3"))  // 32-voxel items, 6 x the fp32 GEMM it computes
    return 6 * 2.0 * ceil((double)out.n * out.t * out.h * out.w / 32.0) * 32.0 * c.cout_p * (double)c.Kp * 1e-9;
  if (!strcmp(kname, "conv_twalk_bf16"))  // 32-pixel columns; 3T - 2 taps per output column (clip ends)
    return 2.0 * out.n * ((out.h * out.w + 31) / 32 * 32) * (double)c.cout_p * c.cin_p * (3.0 * out.t - 2.0) * 1e-9;
  if (!strcmp(kname, "conv_patch32_bf16"))  // 4 frames x 8x8-pixel tiles
    return 2.0 * out.n * ((out.t + 3) / 4 * 4) * (double)((out.h + 7) / 8 * 8) * ((out.w + 7) / 8 * 8) * c.cout_p *
           (double)c.Kp * 1e-9;
  const double m = (double)out.n * out.t * out.h * out.w;
  // conv_dma_x3: six bf16 products per product of the fp32 GEMM it computes (K padded to 32-deep pairs)
  if (!strcmp(kname, "conv_dma_x3"))
    return 6 * 2.0 * (ceil(m / 128.0) * 128.0) * c.cout_p * (double)((c.Kp + 31) / 32 * 32) * 1e-9;
  return 2.0 * (ceil(m / 128.0) * 128.0) * c.cout_p * (double)c.Kp * 1e-9;
}

// Conv parameters of c over an input of shape `in` (output shape in `out`; tensors unset).
ConvParams conv_params(const Conv& c, const Shape5& in, Shape5& out) {
  out.n = in.n;
  out.t = (in.t + 2 * c.pt - c.kt) / c.st + 1;
  out.h = (in.h + 2 * c.ph - c.kh) / c.sh + 1;
  out.w = (in.w + 2 * c.pw - c.kw) / c.sw + 1;
  out.c = c.cout_p;
  ConvParams p{};
  p.w = c.dw;
  p.bias = c.db;
  p.N = in.n, p.Ti = in.t, p.Hi = in.h, p.Wi = in.w, p.Cin = in.c;
  p.To = out.t, p.Ho = out.h, p.Wo = out.w, p.Cout = out.c;
  p.KT = c.kt, p.KH = c.kh, p.KW = c.kw, p.st = c.st, p.sh = c.sh, p.sw = c.sw, p.pt = c.pt, p.ph = c.ph, p.pw = c.pw;
  p.K = c.K, p.Kp = c.Kp;
  p.M = out.n * out.t * out.h * out.w;
  p.Cin2 = c.cin2;
  p.stem = c.stem;
  p.in_bf16 = c.in_bf16;
  p.out_bf16 = c.out_bf16;
  return p;
}

// The kernel run_conv launches for c with parameters p (p.vflags selects A/B variants).
const char* pick_kernel(const Conv& c, ConvParams p) {
  // 7x7 maps (layer4 at 112x112 clips): the split-bf16 direct GEMM beats F(4x4)'s partial edge tiles
  // (convbench 0.284 vs 0.312 ms per 1152-channel launch, profiles/r03p_dma_x3_tiles.txt); per-clip
  // shape rule
  if (c.dwino4 && c.dx3 && p.Ho * p.Wo <= 64 && !p.y_c8 && dma_x3_supported(p)) return "conv_dma_x3";
  const int no4 = p.vflags & (CLASFV_VARIANT_NO_WINO4 | CLASFV_VARIANT_NO_WINO4W);
  if (c.dwino4r && !no4 && !(p.vflags & CLASFV_VARIANT_NO_WINO4R) && wino4r_supported(p)) return "conv_wino4r";
  if (c.dwino4w && !no4 && wino4w_supported(p)) return "conv_wino4w";
  if (c.dwino4 && !(p.vflags & CLASFV_VARIANT_NO_WINO4) && wino4_supported(p)) return "conv_wino4";
  if (c.dwino) {
    const bool no_patch = (p.vflags & CLASFV_VARIANT_NO_WINO_PATCH) != 0;
    if (!no_patch && winoq_supported(p)) return "conv_wino_q";
    if (wino_supported(p)) return "conv_wino";
  }
  if (c.dws16 && !(p.vflags & CLASFV_VARIANT_NO_STEM_BF16) && stem_bf16_supported(p)) return "conv_stem_bf16";
  if (c.dws16 && stem_x3_supported(p)) return "conv_stem_x3";
  // temporal convs on <= 256-voxel clip maps (layer4, T = 4): split-K 4 on the split-bf16 direct GEMM
  // beats the one-tile-row F(4,3) form (convbench 0.119 vs 0.145 ms with both split sums)
  if (c.dwinot && c.dx3 && (long)p.To * p.Ho * p.Wo <= 256 && !p.x_c8 && !p.y_c8 && dma_x3_supported(p))
    return "conv_dma_x3";
  if (c.dwinot && winot_supported(p)) return "conv_winot";
  if (c.dx3 && !(p.vflags & CLASFV_VARIANT_NO_PROJ_X3) && proj_x3_supported(p)) return "conv_proj_x3";
  if (!(p.vflags & (CLASFV_VARIANT_NO_PATCH_BF16 | CLASFV_VARIANT_NO_PATCH32)) && patch32_bf16_supported(p))
    return "conv_patch32_bf16";
  if (!(p.vflags & (CLASFV_VARIANT_NO_PATCH_BF16 | CLASFV_VARIANT_NO_TWALK)) && twalk_bf16_supported(p))
    return "conv_twalk_bf16";
  if (!(p.vflags & CLASFV_VARIANT_NO_PATCH_BF16) && patch_bf16_supported(p)) return "conv_patch_bf16";
  if (c.dx3 && dma_x3_supported(p)) return "conv_dma_x3";
  if (c.stem) return "conv_stem_f32";
  // bf16 direct convs with whole 128-B tap rows (launch_dma takes conv_dma_w at the 128-row M tile)
  return dma_w_ok(p) ? "conv_dma_w" : "conv_dma";
}

// Whether the mid tensor between producer `a` (input shape `in`) and consumer `b` goes through HBM
// in the 8-channel-blocked layout: `a` runs on a kernel that writes it and `b` on conv_winot5,
// which reads it (CLASFV_VARIANT_NO_C8: always channels-last).
bool c8_pair(const Conv& a, const Conv& b, const Shape5& in, const Tuning& tu) {
  if (tu.vflags & CLASFV_VARIANT_NO_C8) return false;
  Shape5 mid, out;
  ConvParams pa = conv_params(a, in, mid);
  ConvParams pb = conv_params(b, mid, out);
  pa.w = a.dwino4w ? (const void*)a.dwino4w : a.dwino4 ? (const void*)a.dwino4 : a.dwino ? (const void*)a.dwino : a.dw;
  pb.w = b.dwinot;
  pa.vflags = pb.vflags = tu.vflags;
  const char* ka = pick_kernel(a, pa);
  // Measured per producer (30 clips, profiles/r02j_*): stem and conv_wino_q (layer1, layer2) write
  // the blocked layout at no cost while the temporal kernels after them gain 7-24 %; conv_wino
  // (layer3) broke even and stays channels-last.
  const bool writes = !strcmp(ka, "conv_wino4") || !strcmp(ka, "conv_wino4w") || !strcmp(ka, "conv_wino4r") ||
                      !strcmp(ka, "conv_wino_q") ||
                      !strcmp(ka, "conv_stem_f32") ||
                      !strcmp(ka, "conv_stem_x3");
  return writes && !a.out_bf16 && !strcmp(pick_kernel(b, pb), "conv_winot") && winot_c8_ok(pb);
}

int run_conv(const Conv& c, const void* x, const Shape5& in, void* y, Shape5& out, const void* res, bool relu,
             hipStream_t s, const void* zero_block, const void* x2, const char** kname, const Tuning& tu, int x_c8 = 0,
             int y_c8 = 0, void* scratch = nullptr, size_t scratch_bytes = 0) {
  if (in.c != c.cin_p) return fail(CLASFV_EINVAL, "internal: channel mismatch");
  ConvParams p = conv_params(c, in, out);
  p.vflags = tu.vflags;
  p.patch_nt = tu.patch_nt;
  p.x = x;
  p.res = res;
  p.y = y;
  p.relu = relu ? 1 : 0;
  p.zero = zero_block;
  p.x2 = x2;
  p.x_c8 = x_c8;
  p.y_c8 = y_c8;
  const char* k = pick_kernel(c, p);
  *kname = k;
  const bool c8_out = !strcmp(k, "conv_wino4") || !strcmp(k, "conv_wino4w") || !strcmp(k, "conv_wino4r") ||
                      !strcmp(k, "conv_wino_q") ||
                      !strcmp(k, "conv_stem_f32") ||
                      !strcmp(k, "conv_stem_x3");
  if ((y_c8 && !c8_out) || (x_c8 && strcmp(k, "conv_winot")))
    return fail(CLASFV_EINVAL, "internal: 8-channel-blocked layout on an unsupported kernel");
  if (!strcmp(k, "conv_wino4r")) {
    p.w = c.dwino4r;
    HIP_TRY(launch_wino4r(p, s));
  } else if (!strcmp(k, "conv_wino4w")) {
    p.w = c.dwino4w;
    HIP_TRY(launch_wino4w(p, s));
  } else if (!strcmp(k, "conv_wino4")) {
    p.w = c.dwino4;
    HIP_TRY(launch_wino4(p, s));
  } else if (!strcmp(k, "conv_wino_q")) {
    p.w = c.dwino;
    HIP_TRY(launch_winoq(p, s));
  } else if (!strcmp(k, "conv_wino")) {
    p.w = c.dwino;
    HIP_TRY(launch_wino(p, s));
  } else if (!strcmp(k, "conv_stem_bf16")) {
    p.w = c.dws16;
    HIP_TRY(launch_stem_bf16(p, s));
  } else if (!strcmp(k, "conv_stem_x3")) {
    p.w = c.dws16;
    HIP_TRY(launch_stem_x3(p, s));
  } else if (!strcmp(k, "conv_winot")) {
    p.w = c.dwinot;
    // split-K on the smallest maps (per-clip shape rule), partial sums in the caller's scratch
    const int S = winot_split_for(p);
    if (S > 1 && scratch && (size_t)S * p.M * p.Cout * sizeof(float) <= scratch_bytes) {
      p.part = reinterpret_cast<float*>(scratch);
      p.n_split = S;
    }
    HIP_TRY(launch_winot(p, s));
  } else if (!strcmp(k, "conv_patch_bf16")) {
    HIP_TRY(launch_patch_bf16(p, s));
  } else if (!strcmp(k, "conv_patch32_bf16")) {
    HIP_TRY(launch_patch32_bf16(p, s));
  } else if (!strcmp(k, "conv_twalk_bf16")) {
    HIP_TRY(launch_twalk_bf16(p, s));
  } else if (!strcmp(k, "conv_proj_x3")) {
    p.w = c.dx3;
    HIP_TRY(launch_proj_x3(p, s));
  } else if (!strcmp(k, "conv_dma_x3")) {
    p.w = c.dx3;
    const int S = dma_split_for(p, 2);
    if (S > 1 && scratch && (size_t)S * p.M * p.Cout * sizeof(float) <= scratch_bytes) {
      p.part = reinterpret_cast<float*>(scratch);
      p.n_split = S;
    }
    HIP_TRY(launch_dma_x3(p, dma_x3_bn(c.cout_p), s));
  } else {
    int mt = 2, bn = c.cout_p;  // stem: one N tile (48 fp32 / 64 bf16 channels)
    if (!c.stem) {
      conv_pick_tile(p.M, c.cout_p, tu.conv_nt, &mt, &bn);
      // split-K on the smallest maps (per-clip shape rule), partial sums in the caller's scratch
      const int S = dma_split_for(p, mt);
      if (S > 1 && scratch && (size_t)S * p.M * p.Cout * sizeof(float) <= scratch_bytes) {
        p.part = reinterpret_cast<float*>(scratch);
        p.n_split = S;
      }
    }
    HIP_TRY(launch_conv(p, mt, bn, s));
  }
  return CLASFV_OK;
}

// Workspace layout for one (N,T,H,W).
struct Layout {
  size_t off[32];
  size_t total;
};
enum Buf { XIN, S0, X0, MID, TA, DSB, L1A, L1, L2A, L2, L3A, L3, L4A, L4, P01, PP2, PP3, PP4, DIDX, NBUF };

void make_layout(int N, int T, int H, int W, Layout& L) {
  const size_t T1 = T, H2 = H / 2, W2 = W / 2;
  size_t sz[NBUF];
  sz[XIN] = (size_t)N * T * H * W * 4;
  sz[S0] = (size_t)N * T1 * H2 * W2 * 48;
  sz[X0] = (size_t)N * T1 * H2 * W2 * 64;
  const size_t l1 = (size_t)N * T1 * H2 * W2 * 64;
  const size_t l2 = (size_t)N * (T / 2) * (H / 4) * (W / 4) * 128;
  const size_t l3 = (size_t)N * (T / 4) * (H / 8) * (W / 8) * 256;
  const size_t l4 = (size_t)N * (T / 8) * (H / 16) * (W / 16) * 512;
  size_t mid = (size_t)N * T1 * H2 * W2 * 144;
  mid = std::max(mid, (size_t)N * T1 * (H / 4) * (W / 4) * 240);
  mid = std::max(mid, (size_t)N * (T / 2) * (H / 8) * (W / 8) * 480);
  mid = std::max(mid, (size_t)N * (T / 4) * (H / 16) * (W / 16) * 960);
  sz[MID] = mid;
  sz[TA] = std::max(std::max(l1, l2), std::max(l3, l4));
  sz[DSB] = std::max(l2, std::max(l3, l4));
  sz[L1A] = sz[L1] = l1;
  sz[L2A] = sz[L2] = l2;
  sz[L3A] = sz[L3] = l3;
  sz[L4A] = sz[L4] = l4;
  sz[P01] = (size_t)N * T1 * H2 * W2 * 64;
  sz[PP2] = (size_t)N * (T / 2) * (H / 4) * (W / 4) * 64;
  sz[PP3] = (size_t)N * (T / 4) * (H / 8) * (W / 8) * 64;
  sz[PP4] = (size_t)N * (T / 8) * (H / 16) * (W / 16) * 64;
  sz[DIDX] = decoder_index_bytes(T, H, W) / sizeof(float);  // the decoder's source-index table
  size_t o = 0;
  for (int i = 0; i < NBUF; ++i) {
    L.off[i] = o;
    o += (sz[i] * sizeof(float) + 255) / 256 * 256;
  }
  L.total = o;
}

// Record one timing event on s (pool grows on demand); returns its index or -1 on failure.
int tick(clasfv_engine* h, hipStream_t s) {
  if (h->nev == (int)h->evs.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    h->evs.push_back(e);
  }
  if (hipEventRecord(h->evs[h->nev], s) != hipSuccess) return -1;
  return h->nev++;
}

float tap_scale(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

// Makes the handle's device current for the scope of an ABI call and restores the caller's.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

#define DEVICE_GUARD(dev)                                                                       \
  DeviceGuard _guard(dev);                                                                      \
  if (_guard.err != hipSuccess)                                                                 \
    return fail(CLASFV_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(_guard.err))

}  // namespace

extern "C" {

const char* clasfv_last_error(void) { return g_err.c_str(); }
int clasfv_version(void) { return CLASFV_ABI_VERSION; }
#ifndef CLASFV_SOURCE_HASH
#define CLASFV_SOURCE_HASH "unhashed"
#endif
const char* clasfv_source_hash(void) { return "clasfv-source-hash:" CLASFV_SOURCE_HASH; }

int clasfv_create(int device, clasfv_t* out) {
  if (!out) return fail(CLASFV_EINVAL, "null out");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(CLASFV_EINVAL, "bad device index");
  auto* e = new clasfv_engine();
  e->device = device;
  e->tune.vflags = env_variants();
  e->tune.conv_nt = env_int("CLASFV_CONV_NT");
  e->tune.patch_nt = env_int("CLASFV_PATCH_NT");
  build_plan(e);
  *out = e;
  return CLASFV_OK;
}

int clasfv_destroy(clasfv_t h) {
  if (!h) return CLASFV_OK;
  DeviceGuard guard(h->device);
  for (auto& c : h->convs) {
    (void)hipFree(c.dw);
    (void)hipFree(c.db);
    (void)hipFree(c.dwino);
    (void)hipFree(c.dwino4);
    (void)hipFree(c.dwino4w);
    (void)hipFree(c.dwino4r);
    (void)hipFree(c.dwinot);
    (void)hipFree(c.dws16);
    (void)hipFree(c.dx3);
  }
  for (auto& c : h->proj) {
    (void)hipFree(c.dw);
    (void)hipFree(c.dx3);
  }
  for (auto* c : h->ctxs) {
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    (void)hipFree(c->arena);
    delete c;
  }
  (void)hipFree(h->b1);
  (void)hipFree(h->w2);
  (void)hipFree(h->w2x3);
  (void)hipFree(h->b2);
  (void)hipFree(h->wh);
  (void)hipFree(h->bh);
  (void)hipFree(h->zero);
  for (auto e : h->evs) (void)hipEventDestroy(e);
  delete h;
  return CLASFV_OK;
}

int clasfv_param_count(clasfv_t h) { return h ? (int)h->params.size() : CLASFV_EINVAL; }

int clasfv_param_info(clasfv_t h, int i, const char** name, int* ndim, int64_t dims[5]) {
  if (!h || i < 0 || i >= (int)h->params.size()) return fail(CLASFV_EINVAL, "bad param index");
  const Param& p = h->params[i];
  if (name) *name = p.name.c_str();
  if (ndim) *ndim = (int)p.shape.size();
  if (dims)
    for (size_t d = 0; d < p.shape.size(); ++d) dims[d] = p.shape[d];
  return CLASFV_OK;
}

int clasfv_load_param(clasfv_t h, const char* name, const float* data, int64_t numel) {
  if (!h || !name) return fail(CLASFV_EINVAL, "null argument");
  std::string n(name);
  if (n.rfind("module.", 0) == 0) n = n.substr(7);
  auto it = h->index.find(n);
  if (it == h->index.end()) return fail(CLASFV_EINVAL, "unknown parameter: " + n);
  Param& p = h->params[it->second];
  if (n.size() > 20 && n.compare(n.size() - 20, 20, ".num_batches_tracked") == 0) {
    p.loaded = true;
    return CLASFV_OK;
  }
  if (numel != p.numel()) return fail(CLASFV_EINVAL, "size mismatch for " + n);
  if (!data) return fail(CLASFV_EINVAL, "null data");
  p.data.assign(data, data + numel);
  p.loaded = true;
  h->ready = false;
  return CLASFV_OK;
}

int clasfv_finalize(clasfv_t h) {
  if (!h) return fail(CLASFV_EINVAL, "null handle");
  for (const auto& p : h->params)
    if (!p.loaded && p.name.find(".fc.") == std::string::npos)
      return fail(CLASFV_ENOTREADY, "parameter not loaded: " + p.name);
  DEVICE_GUARD(h->device);
  // forwards still in flight on any stream read the weight images replaced below
  HIP_TRY(hipDeviceSynchronize());
  const bool bf16 = h->dtype == CLASFV_DTYPE_BF16;
  for (auto& c : h->convs) layout_conv(c, bf16);
  for (auto& c : h->proj) layout_conv(c, bf16);
  std::vector<double> s, t;
  for (auto& c : h->convs) {
    (void)hipFree(c.dw);
    (void)hipFree(c.db);
    (void)hipFree(c.dwino);
    (void)hipFree(c.dwino4);
    (void)hipFree(c.dwino4w);
    (void)hipFree(c.dwino4r);
    (void)hipFree(c.dwinot);
    (void)hipFree(c.dws16);
    (void)hipFree(c.dx3);
    c.dw = c.dws16 = c.dx3 = nullptr;
    c.db = nullptr;
    c.dwino = c.dwino4 = c.dwino4w = c.dwino4r = c.dwinot = nullptr;
    bn_scale_shift(h, c.bn, c.cout, s, t);
    const auto& w = P(h, c.w + ".weight");
    const int taps = c.kt * c.kh * c.kw;
    const int cin = c.cin;
    int rc = upload_conv(
        c, [&](int o, int ci, int tap) { return w[((size_t)o * cin + ci) * taps + tap]; }, s, t, true);
    if (rc) return rc;
    if (use_wino(c, bf16, h->tune.vflags)) {
      std::vector<double> wf((size_t)c.cout * cin * 9);
      for (int o = 0; o < c.cout; ++o)
        for (size_t i = 0; i < (size_t)cin * 9; ++i) wf[(size_t)o * cin * 9 + i] = (double)w[(size_t)o * cin * 9 + i] * s[o];
      std::vector<float> u((size_t)16 * c.cin_p * c.cout_p);
      wino_transform_weights(wf.data(), c.cout, cin, c.cout_p, c.cin_p, u.data());
      if ((rc = upload(u, &c.dwino))) return rc;
      if (c.cout_p % 48 == 0 && c.cin_p % 8 == 0) {
        std::vector<float> u4(wino4_weight_floats(c.cin_p, c.cout_p));
        wino4_transform_weights(wf.data(), c.cout, cin, c.cout_p, c.cin_p, u4.data());
        if ((rc = upload(u4, &c.dwino4))) return rc;
      }
      if (c.cin_p % 8 == 0 && wino4w_weight_floats(c.cin_p, c.cout_p)) {
        std::vector<float> uw(wino4w_weight_floats(c.cin_p, c.cout_p));
        wino4w_transform_weights(wf.data(), c.cout, cin, c.cout_p, c.cin_p, uw.data());
        if ((rc = upload(uw, &c.dwino4w))) return rc;
      }
      if (c.cin_p % 8 == 0 && wino4r_weight_floats(c.cin_p, c.cout_p)) {
        std::vector<float> ur(wino4r_weight_floats(c.cin_p, c.cout_p));
        wino4r_transform_weights(wf.data(), c.cout, cin, c.cout_p, c.cin_p, ur.data());
        if ((rc = upload(ur, &c.dwino4r))) return rc;
      }
    }
    if (!bf16 && c.stem && c.cout_p == 48 && c.kh == 7 && c.kw == 7 && cin <= 4) {  // conv_stem_x3's pieces
      const size_t img = (size_t)48 * 7 * 8 * 4;
      std::vector<float> ws(3 * img, 0.f);  // hi, mid, lo: bf16 of the remainder, in double
      for (int o = 0; o < c.cout; ++o)
        for (int ci = 0; ci < cin; ++ci)
          for (int kh = 0; kh < 7; ++kh)
            for (int kw = 0; kw < 7; ++kw) {
              double r = (double)(float)((double)w[((size_t)o * cin + ci) * 49 + kh * 7 + kw] * s[o]);
              const size_t k = (((size_t)o * 7 + kh) * 8 + kw) * 4 + ci;
              for (int pc = 0; pc < 3; ++pc) {
                const uint32_t hb = (uint32_t)to_bf16((float)r) << 16;
                float f;
                memcpy(&f, &hb, 4);
                ws[pc * img + k] = f;
                r -= f;
              }
            }
      if ((rc = upload_bf16(ws, &c.dws16))) return rc;
    }
    if (bf16 && c.stem && c.cout_p == 64 && c.kh == 7 && c.kw == 7 && cin <= 4) {  // conv_stem_bf16's K order
      const size_t img = (size_t)64 * 7 * 8 * 4;
      std::vector<float> ws(2 * img, 0.f);  // hi image, then lo = bf16(w - hi)
      for (int o = 0; o < c.cout; ++o)
        for (int ci = 0; ci < cin; ++ci)
          for (int kh = 0; kh < 7; ++kh)
            for (int kw = 0; kw < 7; ++kw) {
              const float v = (float)((double)w[((size_t)o * cin + ci) * 49 + kh * 7 + kw] * s[o]);
              const uint32_t hb = (uint32_t)to_bf16(v) << 16;
              float hi;
              memcpy(&hi, &hb, 4);
              const size_t k = (((size_t)o * 7 + kh) * 8 + kw) * 4 + ci;
              ws[k] = hi;
              ws[img + k] = v - hi;
            }
      if ((rc = upload_bf16(ws, &c.dws16))) return rc;
    }
    if (use_winot(c, bf16, h->tune.vflags)) {
      std::vector<double> wf((size_t)c.cout * cin * 3);
      for (int o = 0; o < c.cout; ++o)
        for (size_t i = 0; i < (size_t)cin * 3; ++i) wf[(size_t)o * cin * 3 + i] = (double)w[(size_t)o * cin * 3 + i] * s[o];
      std::vector<float> u((size_t)6 * c.cin_p * c.cout_p);
      winot_transform_weights(wf.data(), c.cout, cin, c.cout_p, c.cin_p, u.data());
      if ((rc = upload(u, &c.dwinot))) return rc;
    }
  }
  // comb_1 + BN1 folded, split per tap (concat order stem, layer1, layer2, layer3, layer4)
  bn_scale_shift(h, "comb_batch_norm_1", 64, s, t);
  const auto& w1 = P(h, "comb_1_layer.weight");
  const auto& bias1 = P(h, "comb_1_layer.bias");
  std::vector<double> zero(64, 0.0);
  const int col0[5] = {0, 64, 128, 256, 512};
  for (int i = 0; i < 5; ++i) {
    if (i == 1) continue;  // folded into the dual proj[0]
    Conv& c = h->proj[i];
    (void)hipFree(c.dw);
    (void)hipFree(c.dx3);
    c.dw = c.dx3 = nullptr;
    const int o0 = col0[i];
    const int kin = c.cin + c.cin2;
    Conv tmp = c;  // upload_conv walks cin: give it the concatenated width
    tmp.cin = tmp.cin_p = kin;
    int rc = upload_conv(
        tmp, [&](int o, int ci, int) { return w1[(size_t)o * 1024 + o0 + ci]; }, s, zero, false);
    if (rc) return rc;
    c.dw = tmp.dw;
    c.dx3 = tmp.dx3;
  }
  std::vector<float> b1(64);
  for (int o = 0; o < 64; ++o) b1[o] = (float)(s[o] * (double)bias1[o] + t[o]);
  bn_scale_shift(h, "comb_batch_norm_2", 64, s, t);
  const auto& w2 = P(h, "comb_2_layer.weight");
  const auto& bias2 = P(h, "comb_2_layer.bias");
  std::vector<float> w2f(64 * 64), b2(64);
  for (int o = 0; o < 64; ++o) {
    for (int k = 0; k < 64; ++k) w2f[o * 64 + k] = (float)((double)w2[o * 64 + k] * s[o]);
    b2[o] = (float)(s[o] * (double)bias2[o] + t[o]);
  }
  const auto& ws = P(h, "segmentation_head.weight");
  const auto& bs = P(h, "segmentation_head.bias");
  const auto& wm = P(h, "motion_head.weight");
  const auto& bm = P(h, "motion_head.bias");
  std::vector<float> whf(8 * 64, 0.f), bhf(8, 0.f);
  for (int k = 0; k < 64; ++k) {
    whf[0 * 64 + k] = ws[k];
    whf[1 * 64 + k] = ws[64 + k];
    for (int m = 0; m < 4; ++m) whf[(2 + m) * 64 + k] = wm[m * 64 + k];
  }
  bhf[0] = bs[0];
  bhf[1] = bs[1];
  for (int m = 0; m < 4; ++m) bhf[2 + m] = bm[m];
  for (float** d : {&h->b1, &h->w2, &h->b2, &h->wh, &h->bh}) {
    (void)hipFree(*d);
    *d = nullptr;
  }
  // W2 and the head weights as hi + mid + lo bf16 pieces in the X3 decoder's lane order
  std::vector<uint16_t> w2x3(DECODER_X3_ELEMS);
  decoder_x3_weights(w2f.data(), whf.data(), w2x3.data());
  (void)hipFree(h->w2x3);
  h->w2x3 = nullptr;
  int rc = upload(b1, &h->b1);
  if (!rc) rc = upload(w2f, &h->w2);
  if (!rc && hipMalloc(&h->w2x3, w2x3.size() * sizeof(uint16_t)) != hipSuccess) rc = fail(CLASFV_EHIP, "hipMalloc");
  if (!rc && hipMemcpy(h->w2x3, w2x3.data(), w2x3.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(CLASFV_EHIP, "hipMemcpy");
  if (!rc) rc = upload(b2, &h->b2);
  if (!rc) rc = upload(whf, &h->wh);
  if (!rc) rc = upload(bhf, &h->bh);
  if (rc) return rc;
  if (!h->zero) {
    HIP_TRY(hipMalloc(&h->zero, 256));
    HIP_TRY(hipMemset(h->zero, 0, 256));
  }
  HIP_TRY(hipDeviceSynchronize());
  h->ready = true;
  return CLASFV_OK;
}

int64_t clasfv_workspace_bytes(clasfv_t h) {
  if (!h) return 0;
  int64_t b = 0;
  for (auto* c : h->ctxs) b += (int64_t)c->arena_bytes;
  return b;
}

int clasfv_set_compute_dtype(clasfv_t h, int dtype) {
  if (!h) return fail(CLASFV_EINVAL, "null handle");
  if (dtype != CLASFV_DTYPE_FP32 && dtype != CLASFV_DTYPE_BF16) return fail(CLASFV_EINVAL, "unknown dtype");
  if (dtype != h->dtype) {
    h->dtype = dtype;
    h->ready = false;  // weights must be re-laid-out: call clasfv_finalize again
  }
  return CLASFV_OK;
}

int clasfv_get_compute_dtype(clasfv_t h) { return h ? h->dtype : CLASFV_EINVAL; }

int clasfv_set_kernel_variants(clasfv_t h, int flags) {
  if (!h) return fail(CLASFV_EINVAL, "null handle");
  if (flags & ~kVariantMask) return fail(CLASFV_EINVAL, "unknown kernel-variant bit");
  if ((flags ^ h->tune.vflags) & CLASFV_VARIANT_NO_WINOGRAD) h->ready = false;  // weight images change
  h->tune.vflags = flags;
  return CLASFV_OK;
}

int clasfv_get_kernel_variants(clasfv_t h) { return h ? h->tune.vflags : CLASFV_EINVAL; }

int clasfv_forward(clasfv_t h, const float* x, int N, int T, int H, int W, float* seg, float* mot, void* stream) {
  if (!h) return fail(CLASFV_EINVAL, "null handle");
  if (!h->ready) return fail(CLASFV_ENOTREADY, "clasfv_finalize has not been called");
  if (!x || !seg || !mot) return fail(CLASFV_EINVAL, "null tensor");
  if (N < 1 || T < 8 || H < 16 || W < 16 || T % 8 || H % 16 || W % 16)
    return fail(CLASFV_EBADSHAPE, "shape must satisfy T % 8 == 0, H % 16 == 0, W % 16 == 0 (got T=" +
                                      std::to_string(T) + " H=" + std::to_string(H) + " W=" + std::to_string(W) + ")");
  hipStream_t s = (hipStream_t)stream;
  DEVICE_GUARD(h->device);
  Layout L;
  make_layout(N, T, H, W, L);
  // this stream's context: created on first use; past kMaxCtx streams the least recently used one is
  // taken over once the device is idle (no queued work can still be using its arena)
  clasfv_engine::Ctx* cx = nullptr;
  for (auto* c : h->ctxs)
    if (c->stream == s) cx = c;
  if (!cx) {
    constexpr size_t kMaxCtx = 4;
    if (h->ctxs.size() < kMaxCtx) {
      cx = new clasfv_engine::Ctx();
      h->ctxs.push_back(cx);
    } else {
      HIP_TRY(hipDeviceSynchronize());
      cx = h->ctxs.front();
      for (auto* c : h->ctxs)
        if (c->last_use < cx->last_use) cx = c;
    }
    cx->stream = s;
  }
  cx->last_use = ++h->ctx_clock;
  if (L.total > cx->arena_bytes) {
    // The arena may still be in use by work queued earlier on its stream.
    HIP_TRY(hipDeviceSynchronize());
    (void)hipFree(cx->arena);
    cx->arena = nullptr;
    cx->arena_bytes = 0;
    HIP_TRY(hipMalloc(&cx->arena, L.total));
    cx->arena_bytes = L.total;
  }
  char* const arena = cx->arena;
  auto buf = [&](int b) { return reinterpret_cast<void*>(arena + L.off[b]); };
  int last_ev = h->ktime ? tick(h, s) : -1;
  auto timed = [&](const char* name, double gflop, double xgflop) {
    if (last_ev < 0) return;
    const int e = tick(h, s);
    if (e >= 0) h->recs.push_back({name, gflop, xgflop, last_ev, e});
    last_ev = e;
  };
  // scratch for a temporal conv reading MID: the rest of MID past its input
  const size_t mid_bytes = L.off[MID + 1] - L.off[MID];
  if (!cx->side) {
    HIP_TRY(hipStreamCreateWithFlags(&cx->side, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&cx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&cx->ev_join, hipEventDisableTiming));
  }
  // Once work is forked to the side stream, every exit of this call (the error returns included)
  // leaves s ordered after everything queued there, so the caller's next use of the arena or the
  // outputs cannot race the projections.
  struct SideJoin {
    clasfv_engine::Ctx* cx;
    hipStream_t s;
    bool pending = false;
    hipError_t join() {
      if (!pending) return hipSuccess;
      pending = false;
      hipError_t e = hipEventRecord(cx->ev_join, cx->side);
      return e != hipSuccess ? e : hipStreamWaitEvent(s, cx->ev_join, 0);
    }
    ~SideJoin() { (void)join(); }
  } side_join{cx, s};
  // a decoder projection on the side stream once its tap is complete on s (timed with its own events;
  // with kernel timing on, the layer4 launches on s run concurrently with these, so their event
  // intervals overlap: the per-kernel sums of a forward exceed its wall time by about the overlap)
  auto run_side = [&](const Conv& c, const void* xin, const Shape5& in, void* y, Shape5& out, const void* x2) {
    HIP_TRY(hipEventRecord(cx->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(cx->side, cx->ev_fork, 0));
    side_join.pending = true;
    const int e0 = h->ktime ? tick(h, cx->side) : -1;
    const char* kname = "";
    int rc_ = run_conv(c, xin, in, y, out, nullptr, false, cx->side, h->zero, x2, &kname, h->tune);
    if (!rc_ && e0 >= 0) {
      const int e1 = tick(h, cx->side);
      if (e1 >= 0) h->recs.push_back({kname, conv_gflop(c, out), conv_exec_gflop(c, out, kname), e0, e1});
    }
    return rc_;
  };
  auto run = [&](const Conv& c, const void* xin, const Shape5& in, void* y, Shape5& out, const void* res, bool relu,
                 const void* x2 = nullptr, int x_c8 = 0, int y_c8 = 0) {
    const char* kname = "";
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    if (xin == buf(MID)) {
      const size_t used = ((size_t)in.n * in.t * in.h * in.w * in.c * sizeof(float) + 255) / 256 * 256;
      if (used < mid_bytes) {
        scratch = arena + L.off[MID] + used;
        scratch_bytes = mid_bytes - used;
      }
    }
    int rc_ = run_conv(c, xin, in, y, out, res, relu, s, h->zero, x2, &kname, h->tune, x_c8, y_c8, scratch,
                       scratch_bytes);
    if (!rc_) timed(kname, conv_gflop(c, out), conv_exec_gflop(c, out, kname));
    return rc_;
  };

  HIP_TRY(launch_pack_input(x, reinterpret_cast<float*>(buf(XIN)), N, T, H * W, s));
  timed("pack_input_kernel", 0.0, 0.0);
  Shape5 sx{N, T, H, W, 4}, s0, sx0;
  Shape5 sp, sp2, sp3, sp4;  // decoder tap projections
  int rc;
  size_t ci = 0;
  // Conv2Plus1D mid tensors (and the stem's) are 8-channel-blocked where c8_pair allows
  const int c8s = c8_pair(h->convs[0], h->convs[1], sx, h->tune);
  if ((rc = run(h->convs[ci++], buf(XIN), sx, buf(S0), s0, nullptr, true, nullptr, 0, c8s))) return rc;
  if ((rc = run(h->convs[ci++], buf(S0), s0, buf(X0), sx0, nullptr, true, nullptr, c8s, 0))) return rc;
  const int outs[4][2] = {{L1A, L1}, {L2A, L2}, {L3A, L3}, {L4A, L4}};
  void* cur = buf(X0);
  Shape5 cs = sx0, taps_shape[5];
  void* taps[5];
  taps[0] = cur;
  taps_shape[0] = cs;
  for (int li = 0; li < 4; ++li) {
    for (int b = 0; b < 2; ++b) {
      const Conv& sp1 = h->convs[ci++];
      const Conv& tp1 = h->convs[ci++];
      const Conv& sp2 = h->convs[ci++];
      const Conv& tp2 = h->convs[ci++];
      const Conv* ds = (ci < h->convs.size() && h->convs[ci].role == DS) ? &h->convs[ci++] : nullptr;
      Shape5 sm, sa, sm2, so, sd;
      const int c8a = c8_pair(sp1, tp1, cs, h->tune);
      if ((rc = run(sp1, cur, cs, buf(MID), sm, nullptr, true, nullptr, 0, c8a))) return rc;
      if ((rc = run(tp1, buf(MID), sm, buf(TA), sa, nullptr, true, nullptr, c8a, 0))) return rc;
      const int c8b = c8_pair(sp2, tp2, sa, h->tune);
      if ((rc = run(sp2, buf(TA), sa, buf(MID), sm2, nullptr, true, nullptr, 0, c8b))) return rc;
      const void* res = cur;
      if (ds) {
        if ((rc = run(*ds, cur, cs, buf(DSB), sd, nullptr, false))) return rc;
        res = buf(DSB);
      }
      void* out = buf(outs[li][b]);
      if ((rc = run(tp2, buf(MID), sm2, out, so, res, true, nullptr, c8b, 0))) return rc;
      cur = out;
      cs = so;
    }
    taps[li + 1] = cur;
    taps_shape[li + 1] = cs;
    // decoder projections at tap resolution (P01 = W0 f0 + W1 f1, P2, P3) on the side stream while
    // layer4 runs: its convs (600-920 blocks for 30 clips, 1.2-1.8 rounds of the chip's block slots)
    // leave CUs idle that the projections fill (forked earlier, P01 only shared layer2's full grids:
    // r03i trace, no gain); P4 after layer4 on s
    if (li == 2) {
      if ((rc = run_side(h->proj[0], taps[0], taps_shape[0], buf(P01), sp, taps[1]))) return rc;
      if ((rc = run_side(h->proj[2], taps[2], taps_shape[2], buf(PP2), sp2, nullptr))) return rc;
      if ((rc = run_side(h->proj[3], taps[3], taps_shape[3], buf(PP3), sp3, nullptr))) return rc;
    }
  }
  if ((rc = run(h->proj[4], taps[4], taps_shape[4], buf(PP4), sp4, nullptr, false))) return rc;
  HIP_TRY(side_join.join());  // the side stream's projections are complete before the decoder

  DecParams d{};
  const Shape5 tsh[4] = {sp, sp2, sp3, sp4};
  const int tb[4] = {P01, PP2, PP3, PP4};
  for (int i = 0; i < 4; ++i) {
    d.tap[i].p = reinterpret_cast<const float*>(buf(tb[i]));
    d.tap[i].T = tsh[i].t;
    d.tap[i].H = tsh[i].h;
    d.tap[i].W = tsh[i].w;
    d.tap[i].st = tap_scale(tsh[i].t, T);
    d.tap[i].sh = tap_scale(tsh[i].h, H);
    d.tap[i].sw = tap_scale(tsh[i].w, W);
  }
  d.b1 = h->b1;
  d.w2 = h->w2;
  d.b2 = h->b2;
  d.wh = h->wh;
  d.bh = h->bh;
  d.seg = seg;
  d.mot = mot;
  d.N = N, d.T = T, d.H = H, d.W = W;
  d.bf16 = h->dtype == CLASFV_DTYPE_BF16 && !(h->tune.vflags & CLASFV_VARIANT_NO_DECODER_BF16);
  d.w2x3 = h->w2x3;
  d.x3 = h->dtype != CLASFV_DTYPE_BF16 && !(h->tune.vflags & CLASFV_VARIANT_NO_DECODER_X3);
  d.idx = buf(DIDX);
  HIP_TRY(launch_decoder(d, s));
  // comb_2 (64x64) and the heads (6 useful of the 16 rows of their MFMA tile) per output voxel, in the
  // products of the pipe they run on: fp32 engines six split-bf16 products each (bf16 pipe), bf16
  // engines three for comb_2 and six for the heads (bf16 pipe), the no_decoder_x3 variant one f32
  // product each (f32 pipe)
  const double dec_px = d.x3 ? 6.0 * (64 * 64 + 64 * 16) : d.bf16 ? 3.0 * 64 * 64 + 6.0 * 64 * 16 : 64 * 64 + 64 * 16;
  timed(d.x3 || d.bf16 ? "decoder_kernel" : "decoder_kernel_f32", 2.0 * N * (double)T * H * W * (64 * 64 + 64 * 6) * 1e-9,
        2.0 * N * (double)T * H * W * dec_px * 1e-9);
  return CLASFV_OK;
}

int clasfv_set_kernel_timing(clasfv_t h, int enable) {
  if (!h) return fail(CLASFV_EINVAL, "null handle");
  h->ktime = enable != 0;
  h->recs.clear();
  h->nev = 0;
  return CLASFV_OK;
}

int clasfv_kernel_timing(clasfv_t h, int cap, const char** names, int* launches, double* ms, double* gflop,
                         double* xgflop) {
  if (!h || cap < 0 || (cap > 0 && (!names || !launches || !ms || !gflop || !xgflop)))
    return fail(CLASFV_EINVAL, "bad argument");
  if (h->nev > 0) HIP_TRY(hipEventSynchronize(h->evs[h->nev - 1]));
  int n = 0;
  for (const auto& r : h->recs) {
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, h->evs[r.e0], h->evs[r.e1]));
    int i = 0;
    while (i < n && strcmp(names[i], r.name) != 0) ++i;
    if (i == n) {
      if (n == cap) return fail(CLASFV_EINVAL, "kernel timing: cap too small");
      names[n] = r.name;
      launches[n] = 0;
      ms[n] = gflop[n] = xgflop[n] = 0.0;
      ++n;
    }
    launches[i] += 1;
    ms[i] += t;
    gflop[i] += r.gflop;
    xgflop[i] += r.xgflop;
  }
  h->recs.clear();
  h->nev = 0;
  return n;
}

int clasfv_build_clips(const float* video, int T, int H, int W, const int32_t* table, int n, int interp, float* clips,
                       void* stream) {
  if (!video || !table || !clips || n < 0 || T < 1 || H < 1 || W < 1) return fail(CLASFV_EINVAL, "bad argument");
  if (n == 0) return CLASFV_OK;
  HIP_TRY(launch_build_clips(video, T, H * W, table, n, interp, clips, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_pass_labels(const float* logits, int K, const int32_t* clip0, int T, int step, int H, int W, int interp,
                       uint8_t* labels, void* stream) {
  if (!logits || !clip0 || !labels || K < 1 || K > CLASFV_MAX_PASSES || T < 1 || step < 1)
    return fail(CLASFV_EINVAL, "bad argument (K must be in [1, 64])");
  HIP_TRY(launch_pass_labels(logits, K, clip0, T, step, H * W, interp, 0, labels, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_pass_labels_margin(const float* margin, int K, const int32_t* clip0, int T, int step, int H, int W,
                              int interp, uint8_t* labels, void* stream) {
  if (!margin || !clip0 || !labels || K < 1 || K > CLASFV_MAX_PASSES || T < 1 || step < 1)
    return fail(CLASFV_EINVAL, "bad argument (K must be in [1, 64])");
  HIP_TRY(launch_pass_labels(margin, K, clip0, T, step, H * W, interp, 1, labels, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_logit_margin(const float* logits, int n, int H, int W, float* margin, void* stream) {
  if (!logits || !margin || n < 0 || H < 1 || W < 1) return fail(CLASFV_EINVAL, "bad argument");
  if (n == 0) return CLASFV_OK;
  HIP_TRY(launch_logit_margin(logits, n, H * W, margin, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_fuse_votes(const uint8_t* labels, int K, int T, int step, int H, int W, int method, uint8_t* fused,
                      void* stream) {
  if (!labels || !fused || K < 1 || K > CLASFV_MAX_PASSES || T < 1 || step < 1 || T - (step - 1) < 1)
    return fail(CLASFV_EINVAL, "bad argument (K must be in [1, 64])");
  const int m = method & ~CLASFV_FUSE_FORCE_GENERIC;
  if (m != CLASFV_FUSE_MAJORITY && m != CLASFV_FUSE_SIMPLE && m != CLASFV_FUSE_STAPLE && m != CLASFV_FUSE_ITKVOTING)
    return fail(CLASFV_EINVAL, "unknown method");
  HIP_TRY(launch_fuse_votes(labels, K, T, step, H * W, method, fused, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_warp(const float* img, int N, int C, int H, int W, const float* motion, int64_t m_sn, int64_t m_sc,
                float* out, void* stream) {
  if (!img || !motion || !out || N < 1 || C < 1 || H < 1 || W < 1) return fail(CLASFV_EINVAL, "bad argument");
  HIP_TRY(launch_warp(img, N, C, H, W, motion, m_sn, m_sc, out, (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_warp_backward(const float* grad_out, const float* img, int N, int C, int H, int W, const float* motion,
                         int64_t m_sn, int64_t m_sc, float* grad_img, float* grad_motion, void* stream) {
  if (!grad_out || !img || !motion || (!grad_img && !grad_motion) || N < 1 || C < 1 || H < 1 || W < 1)
    return fail(CLASFV_EINVAL, "bad argument");
  HIP_TRY(launch_warp_backward(grad_out, img, N, C, H, W, motion, m_sn, m_sc, grad_img, grad_motion,
                               (hipStream_t)stream));
  return CLASFV_OK;
}

int clasfv_preprocess_video(const uint8_t* frames, int T, int Hs, int Ws, int H, int W, float* out, void* stream) {
  if (!frames || !out || T < 1 || Hs < 1 || Ws < 1 || H < 1 || W < 1 || H > 65535 || T > 65535)
    return fail(CLASFV_EINVAL, "bad argument");
  HIP_TRY(launch_preprocess_video(frames, T, Hs, Ws, H, W, out, (hipStream_t)stream));
  return CLASFV_OK;
}

int64_t clasfv_zeroone_workspace_bytes(void) { return (int64_t)sizeof(float) * zeroone_partials_floats(); }

int clasfv_zeroone_normalize(float* video, int64_t n, float* workspace, void* stream) {
  if (!video || !workspace || n < 1) return fail(CLASFV_EINVAL, "bad argument");
  HIP_TRY(launch_zeroone_normalize(video, n, workspace, (hipStream_t)stream));
  return CLASFV_OK;
}

}  // extern "C"
