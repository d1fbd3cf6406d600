// Occupancy / placement probe (not product code): the MFMA issue rate of conv_wino4-shaped blocks.
// Each wave issues CH x 36 v_mfma_f32_16x16x4_f32 on 18 accumulators (the conv_wino4 chunk pattern:
// every accumulator twice per chunk, 6 apart), in blocks of W waves with L bytes of static LDS and
// 168 VGPRs allocated (3 waves per SIMD), over a grid of G blocks.
// usage: occ_probe  -> one line per configuration
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int W, int L, int CH, int VG>
__global__ __launch_bounds__(64 * W) void k(float* out, float seed) {
  __shared__ char smem[L];
  f32x4 acc[18];
  for (int i = 0; i < 18; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a[12], b[36];
  for (int i = 0; i < 12; ++i) a[i] = seed + threadIdx.x * 1e-3f + i;
  for (int i = 0; i < 36; ++i) b[i] = seed - threadIdx.x * 1e-3f - i * 0.5f;
  smem[threadIdx.x] = (char)threadIdx.x;
  for (int c = 0; c < CH; ++c) {
#pragma unroll
    for (int gg = 0; gg < 3; ++gg)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * gg + jj;
            acc[j * 3 + nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2 * j + ks], b[(nt * 3 + gg) * 4 + 2 * jj + ks],
                                                                   acc[j * 3 + nt], 0, 0, 0);
          }
    if (c % 2 == 1) __syncthreads();
  }
  if constexpr (VG == 168) asm volatile("" ::: "v167");
  if constexpr (VG == 128) asm volatile("" ::: "v127");
  float s = smem[(threadIdx.x + 1) % L];
  for (int i = 0; i < 18; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 64 * W + threadIdx.x] = s;
}

template <int W, int L, int CH, int VG>
void run(const char* name, int grid, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<W, L, CH, VG>), dim3(grid), dim3(64 * W), 0, 0, out, 1.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double flop = (double)grid * W * CH * 36 * 2048.0;
  const double ideal = flop / 157.3e12 * 1e3;
  printf("%-44s grid=%6d  %.3f ms  %.1f TFLOP/s  (ideal %.3f ms, %.2f)\n", name, grid, best, flop / best / 1e9, ideal,
         ideal / best);
}

int main() {
  float* out;
  hipMalloc(&out, (size_t)40320 * 768 * 4);
  run<6, 78432, 8, 168>("6 waves, 78 KB LDS, 168 VGPR, 8 chunks", 40320, out);
  run<6, 78432, 80, 168>("6 waves, 78 KB LDS, 168 VGPR, 80 chunks", 4032, out);
  run<6, 50000, 8, 168>("6 waves, 50 KB LDS, 168 VGPR, 8 chunks", 40320, out);
  run<6, 78432, 8, 128>("6 waves, 78 KB LDS, 128 VGPR, 8 chunks", 40320, out);
  run<4, 78432, 12, 168>("4 waves, 78 KB LDS, 168 VGPR, 12 chunks", 40320, out);
  run<12, 100000, 8, 168>("12 waves, 100 KB LDS, 168 VGPR, 8 chunks", 20160, out);
  run<12, 100000, 80, 168>("12 waves, 100 KB LDS, 168 VGPR, 80 chunks", 2016, out);
  run<8, 78432, 6, 168>("8 waves, 78 KB LDS, 168 VGPR, 6 chunks", 40320, out);
  return 0;
}
