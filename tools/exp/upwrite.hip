// Experiment (not product code): write throughput of the upconv output pattern vs a linear fill.
#include <hip/hip_runtime.h>
#include <cstdio>
// A: block = 256 threads x float4 over (ox, c) of one row, loop over R rows (upconv_fused layout)
__global__ __launch_bounds__(256) void rows_kernel(float* y, int Ho, int per_row, int chunks, int R) {
  const int chunk = blockIdx.x % chunks, n = blockIdx.x / chunks;
  const int j = chunk * 256 + threadIdx.x;
  if (j >= per_row) return;
  float* p = y + ((size_t)n * Ho * per_row + j) * 4;
  for (int oy = 0; oy < R; ++oy) {
    float v = (float)(oy + j);
    *reinterpret_cast<float4*>(p + (size_t)oy * per_row * 4) = make_float4(v, v, v, v);
  }
}
// B: one row per block-iteration, grid-stride over rows (each block writes whole contiguous rows)
__global__ __launch_bounds__(256) void lin_kernel(float4* y, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float v = (float)i;
    y[i] = make_float4(v, v, v, v);
  }
}
// C: rows kernel but R rows interleaved across blocks: block handles (row-block, chunk) with short R
int main() {
  const int B = 64, Ho = 160, Wo = 160, Co = 512;
  const int per_row = Wo * Co / 4, chunks = (per_row + 255) / 256;
  size_t n = (size_t)B * Ho * Wo * Co;
  float* y; hipMalloc(&y, n * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(rows_kernel, dim3(B * chunks), dim3(256), 0, 0, y, Ho, per_row, chunks, Ho);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("rows  R=%d: %.3f ms %.1f GB/s\n", Ho, ms, n * 4 / ms / 1e6);
    for (int g : {1024, 4096, 16384}) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(lin_kernel, dim3(g), dim3(256), 0, 0, (float4*)y, n / 4);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      printf("linear grid %d: %.3f ms %.1f GB/s\n", g, ms, n * 4 / ms / 1e6);
    }
  }
  hipFree(y);
  return 0;
}
