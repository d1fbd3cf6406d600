// HBM write / read / copy rate probe: grid-stride 16-B-per-lane kernels over a buffer of the given
// size (MiB), best of 5 timed rounds of 10 launches. usage: bw_probe MIB
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void wr(f4* y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f4{1.f, 2.f, 3.f, (float)i};
}
__global__ void rd(const f4* x, size_t n, f4* out) {
  f4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += x[i];
  if (acc[0] == 12345.f) out[0] = acc;
}
__global__ void cp(const f4* x, f4* y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = x[i];
}
// blocks each write one contiguous 80-KiB piece (a conv block's output tile), 1 KiB per wave instruction
__global__ void wr_tiles(f4* y, size_t n) {
  const size_t per = 80 * 1024 / 16;
  const size_t b0 = blockIdx.x * per;
  for (size_t i = threadIdx.x; i < per && b0 + i < n; i += blockDim.x) y[b0 + i] = f4{1.f, 2.f, 3.f, (float)i};
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? atoll(argv[1]) : 1024;
  const size_t n = mib * 1024 * 1024 / 16;
  f4 *x, *y;
  CK(hipMalloc(&x, n * 16));
  CK(hipMalloc(&y, n * 16));
  CK(hipMemset(x, 0, n * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 256 * 8;
  for (int k = 0; k < 4; ++k) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a, 0));
      for (int it = 0; it < 10; ++it) {
        if (k == 0) hipLaunchKernelGGL(wr, dim3(grid), dim3(256), 0, 0, y, n);
        if (k == 1) hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, x, n, y);
        if (k == 2) hipLaunchKernelGGL(cp, dim3(grid), dim3(256), 0, 0, x, y, n);
        if (k == 3) hipLaunchKernelGGL(wr_tiles, dim3((unsigned)((n * 16 + 80 * 1024 - 1) / (80 * 1024))), dim3(256), 0, 0, y, n);
      }
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms / 10 < best) best = ms / 10;
    }
    const double bytes = (k == 2 ? 2.0 : 1.0) * n * 16;
    printf("%-9s %zu MiB: %.3f ms  %.2f TB/s\n", k == 0 ? "write" : k == 1 ? "read" : k == 2 ? "copy" : "wr_tiles", mib, best, bytes / best * 1e-9);
  }
  return 0;
}
