// Shared declarations of the CLAS-FV engine (internal; the public ABI is include/clasfv.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "clasfv.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ReLU in one instruction, bit-identical to fmaxf(x, 0.f) for every non-NaN x (-0 and negatives give
// +0): fmaxf compiles to two v_max_f32 (an IEEE canonicalisation of x, then the max)
__device__ inline float relu1(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

// a - b on 4 floats as two packed adds with the second operand negated (exactly a - b per lane): the
// compiler emits four scalar v_sub_f32 for the vector subtraction
__device__ inline f32x4 psub4(f32x4 a, f32x4 b) {
  const f32x2 alo = {a[0], a[1]}, ahi = {a[2], a[3]}, blo = {b[0], b[1]}, bhi = {b[2], b[3]};
  f32x2 lo, hi;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(lo) : "v"(alo), "v"(blo));
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(hi) : "v"(ahi), "v"(bhi));
  return f32x4{lo[0], lo[1], hi[0], hi[1]};
}


// n / d for a runtime divisor d >= 1 and n < 2^31 as one multiply-high and an add (Granlund-Montgomery
// with a 33-bit multiplier): a per-lane integer division by a kernel argument is a ~30-instruction
// VALU sequence, and the block prologues / epilogues of the conv kernels decode tile indices with
// several of them. Exhaustively checked for d < 5000 and sampled up to 2^31 (tools/).
struct FastDiv {
  unsigned m;
  int l;
};
inline FastDiv fast_div(unsigned d) {
  int l = 0;
  while ((1u << l) < d) ++l;
  return FastDiv{(unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
}
__device__ inline int fdiv(int n, FastDiv f) { return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.l); }

// One bias-free conv3d (BN folded into weights/bias) as an implicit GEMM over channels-last
// activations: Y[m][n] = sum_k A[m][k] * W[n][k] (+bias[n], +res[m][n], relu).
//   m = ((n*To + to)*Ho + ho)*Wo + wo            (output voxel)
//   k = ((kt*KH + kh)*KW + kw)*Cin + c           (tap-major, channel-minor)
struct ConvParams {
  const void* x;      // [N][Ti][Hi][Wi][Cin], fp32 or bf16 (in_bf16)
  const void* w;      // [Cout_alloc][Kp], zero padded, same dtype as x
  const float* bias;  // [Cout_alloc] or nullptr
  const void* res;    // [M][Cout] or nullptr (may alias y), dtype of y
  void* y;            // [M][Cout], fp32 or bf16 (out_bf16)
  int N, Ti, Hi, Wi, Cin;
  int To, Ho, Wo, Cout;
  int KT, KH, KW, st, sh, sw, pt, ph, pw;
  int K, Kp, M, relu;
  const void* zero;   // >= 16 zero bytes (source of padding taps for the LDS-DMA path)
  const void* x2;     // optional second input of a 1x1x1 conv (same voxels), K columns after x's
  int Cin2;
  int stem;           // fp32 4-channel input (3 + pad): register-staged kernel, per-float4 tap decode
  int in_bf16, out_bf16;
  // 8-channel-blocked activations [C/8][N*T*H*W][8] instead of channels-last (fp32 only): the
  // mid tensor of a Conv2Plus1D between a stride-1 spatial producer (conv_wino_q on 8x8-pixel
  // patches and conv_stem_f32 write y_c8) and the temporal Winograd consumer (conv_winot5 reads x_c8), whose
  // 8-channel chunks then read whole 128-B lines instead of 32 B of every pixel.
  int x_c8, y_c8;
  // Kernel-choice switches of the engine (CLASFV_VARIANT_* of include/clasfv.h, read from the
  // environment once at clasfv_create or set with clasfv_set_kernel_variants) and the tuning
  // overrides of the bf16 patch kernel's N tile (0: automatic).
  int vflags, patch_nt;
  // Split-K (conv_winot5 on grids smaller than the chip): n_split > 1 blocks per output tile, each
  // over a contiguous range of input-channel chunks, write their partial sums to part[split] (fp32,
  // [n_split][M][Cout]); a second pass adds them in split order with bias, residual and ReLU.
  float* part;
  int n_split;
};

// Decoder tap: low-resolution projection P_i = (s1 * W_i) . f_i, channels-last with 64 channels.
struct DecTap {
  const float* p;
  int T, H, W;
  float st, sh, sw;  // align_corners=True source scales (in-1)/(out-1)
};

struct DecParams {
  DecTap tap[4];      // (stem+layer1), layer2, layer3, layer4
  const float* b1;    // [64]    comb_1 bias with BN1 folded
  const float* w2;    // [64*64] comb_2 weight with BN2 folded, [n][k]
  const void* w2x3;   // fp32 engines: W2 and Wh as three bf16 pieces (hi, mid, lo: w = hi + mid + lo to
                      // 24 bits) in the MFMA lane order, decoder_x3_weights (decoder.hip)
  const float* b2;    // [64]
  const float* wh;    // [8*64]  rows: seg0, seg1, mot0..mot3, 0, 0
  const float* bh;    // [8]
  float* seg;         // (N,2,T,H,W)
  float* mot;         // (N,4,T,H,W)
  int N, T, H, W;
  int bf16;           // comb_2 on bf16 MFMAs (bf16 engines; taps, heads and outputs stay fp32)
  int x3;             // fp32 engines: comb_2 as six bf16 products of 3-way split operands (fp32-accurate)
  void* idx;          // device scratch of decoder_index_bytes(T, H, W): the per-launch source-index table
                      // (launch_decoder fills it on the stream before the decoder reads it)
};
// bytes of DecParams::idx: per tap, T frame + H row + W column entries of 16 B
inline size_t decoder_index_bytes(int T, int H, int W) { return (size_t)4 * (T + H + W) * 16; }

// Launchers (stream-ordered, no synchronisation). Return hipError_t of the launch.
hipError_t launch_conv(const ConvParams& p, int mt, int bn, hipStream_t s);
// Block tile (BM = 64*mt rows, bn output channels) for an M x cout_p conv.
void conv_pick_tile(int M, int cout_p, int force_nt, int* mt, int* bn);
// Fused Winograd F(2x2,3x3) path for stride-1 1x3x3 fp32 convs; p.w = transformed weights.
bool wino_supported(const ConvParams& p);
hipError_t launch_wino(const ConvParams& p, hipStream_t s);
// U[cin_p/8][4][cout_p][4][4][2] from folded weights w[cout][cin][3][3] (double).
void wino_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U);
// Patch-tiled Winograd F(2x2,3x3) for Ho, Wo % 4 == 0 (winograd2.hip); p.w = conv_wino's U.
bool winoq_supported(const ConvParams& p);
hipError_t launch_winoq(const ConvParams& p, hipStream_t s);
// Fused Winograd F(4x4,3x3) for stride-1 1x3x3 fp32 convs without residual (winograd4.hip; partial
// 4x4 tiles at the edges of maps with Ho, Wo % 4 != 0); p.w = wino4_transform_weights' layout.
bool wino4_supported(const ConvParams& p);
hipError_t launch_wino4(const ConvParams& p, hipStream_t s);
// MFMA work (GFLOP) one conv_wino4 launch executes (16 MFMA rows per tile group, padding included).
double wino4_exec_gflop(const ConvParams& p);
// conv_wino4's transformed weights (wino4_weight_floats(cin_p, cout_p) floats) from folded weights
// w[cout][cin][3][3] (double).
void wino4_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U);
size_t wino4_weight_floats(int cin_p, int cout_p);
// conv_wino4 with wide output-channel blocks (16 NTN channels, NTN = wino4w_ntn(cout) in {9, 6, 5}; one
// 4-wave block per CU; winograd4w.hip): the same products and order as conv_wino4, bit-identical.
bool wino4w_supported(const ConvParams& p);
hipError_t launch_wino4w(const ConvParams& p, hipStream_t s);
double wino4w_exec_gflop(const ConvParams& p);
void wino4w_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U);
size_t wino4w_weight_floats(int cin_p, int cout_p);  // 0: no wide block for this cout_p
// conv_wino4r: conv_wino4w's arithmetic on 12 row waves per block (3 per SIMD), its own U layout
bool wino4r_supported(const ConvParams& p);
hipError_t launch_wino4r(const ConvParams& p, hipStream_t s);
double wino4r_exec_gflop(const ConvParams& p);
void wino4r_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U);
size_t wino4r_weight_floats(int cin_p, int cout_p);
// Fused Winograd F(4,3)-in-time path for stride-1 3x1x1 fp32 convs; p.w = transformed weights.
bool winot_supported(const ConvParams& p);
hipError_t launch_winot(const ConvParams& p, hipStream_t s);
// launch_winot would run conv_winot5, the variant that also reads 8-channel-blocked input (x_c8).
bool winot_c8_ok(const ConvParams& p);
// Split-K: y = [relu](sum of p.part[0 .. n_split) in split order + bias + res), fp32 channels-last.
hipError_t launch_split_sum(const ConvParams& p, hipStream_t s);
// Split-K factor for launch_conv's conv_dma with M tile mt (1: no split; per-clip shape only).
int dma_split_for(const ConvParams& p, int mt);
// conv_stem_x3: the fp32 engines' stem on split-bf16 MFMAs (conv.hip)
bool stem_x3_supported(const ConvParams& p);
hipError_t launch_stem_x3(const ConvParams& p, hipStream_t s);
// conv_dma_x3: fp32 implicit GEMM on split-bf16 MFMAs (six products, fp32-accurate; conv.hip)
bool dma_x3_supported(const ConvParams& p);
bool dma_w_ok(const ConvParams& p);
int dma_x3_bn(int cout_p);
hipError_t launch_dma_x3(const ConvParams& p, int bn, hipStream_t s);
void dma_x3_weight_image(const float* w, int cout_alloc, int Kp, uint16_t* out);
size_t dma_x3_weight_elems(int cout_alloc, int Kp);
// Split-K factor (ConvParams::n_split) for launch_winot (1: no split; per-clip shape only); the
// caller provides ConvParams::part with n_split * M * Cout floats.
int winot_split_for(const ConvParams& p);
// U[cin_p/8][6][cout_p/64][64][8] from folded weights w[cout][cin][3] (double).
void winot_transform_weights(const double* w, int cout, int cin, int cout_p, int cin_p, float* U);
// Patch-staged bf16 implicit GEMM for stride-1 1x3x3 and 3x1x1 convs (conv_patch.hip); p.w = conv_dma's
// image.
bool proj_x3_supported(const ConvParams& p);
hipError_t launch_proj_x3(const ConvParams& p, hipStream_t s);
bool patch_bf16_supported(const ConvParams& p);
bool patch32_bf16_supported(const ConvParams& p);
hipError_t launch_patch32_bf16(const ConvParams& p, hipStream_t s);
hipError_t launch_patch_bf16(const ConvParams& p, hipStream_t s);
// Frame-walking bf16 temporal 3x1x1 conv with 64 output channels (twalk.hip; Cin 64 or 160).
bool twalk_bf16_supported(const ConvParams& p);
hipError_t launch_twalk_bf16(const ConvParams& p, hipStream_t s);
// bf16 stem (config[4]): fp32 4-channel clip split into bf16 hi + lo in registers; p.w = hi and lo
// images, each [64][7][8][4] bf16.
bool stem_bf16_supported(const ConvParams& p);
hipError_t launch_stem_bf16(const ConvParams& p, hipStream_t s);
hipError_t launch_decoder(const DecParams& p, hipStream_t s);
constexpr int DECODER_X3_ELEMS = 3 * 4096 + 3 * 1024;  // bf16 values of DecParams::w2x3
void decoder_x3_weights(const float* w2, const float* wh, uint16_t* out);
hipError_t launch_pack_input(const float* x, float* y, int N, int T, int HW, hipStream_t s);
