// Achievable fp32 / bf16 MFMA issue rate on this MI355X (not product code): every wave issues
// ITERS x 24 independent MFMAs (24 accumulators, operands in registers), W waves per SIMD.
// usage: mfma_peak  -> prints TFLOP/s for v_mfma_f32_16x16x4_f32 and v_mfma_f32_16x16x32_bf16
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int BF>
__global__ __launch_bounds__(256) void k(float* out, int iters, float seed) {
  f32x4 acc[24];
  for (int i = 0; i < 24; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a = seed + threadIdx.x * 1e-3f, b = seed - threadIdx.x * 1e-3f;
  bf16x8 ab, bb;
  for (int i = 0; i < 8; ++i) {
    ab[i] = (__bf16)(a + i);
    bb[i] = (__bf16)(b - i);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      if constexpr (BF)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 24; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 8 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int bf = 0; bf < 2; ++bf)
    for (int bpc : {1, 2, 3}) {  // blocks (of 4 waves) per CU -> waves per SIMD
      const int nb = 256 * bpc, iters = bf ? 4000 : 2000;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (bf) hipLaunchKernelGGL(k<1>, dim3(nb), dim3(256), 0, 0, out, iters, 1.f);
        else hipLaunchKernelGGL(k<0>, dim3(nb), dim3(256), 0, 0, out, iters, 1.f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flop = (double)nb * 4 * iters * 24 * (bf ? 16384.0 : 2048.0);
      printf("%s waves/SIMD=%d  %.3f ms  %.1f TFLOP/s\n", bf ? "bf16 16x16x32" : "fp32 16x16x4 ", bpc, ms, flop / ms / 1e9);
    }
  return 0;
}
