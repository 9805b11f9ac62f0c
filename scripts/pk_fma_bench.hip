// Microbenchmark: issue cost of v_fma_f32 vs v_pk_fma_f32 (same FLOPs) on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
#define ITERS 4096
__global__ void k_scalar(float *out, float a, float b) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                 "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
__global__ void k_packed(float *out, float a, float b) {
  f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 2, x2 = x0 + 4, x3 = x0 + 6;
  f2 A = {a, a}, B = {b, b};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(A), "v"(B));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0.x + x0.y + x1.x + x1.y + x2.x + x2.y + x3.x + x3.y;
}
__global__ void k_packed8(float *out, float a, float b) {  // 8 independent packed accumulators
  f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 2, x2 = x0 + 4, x3 = x0 + 6, x4 = x0 + 8, x5 = x0 + 10, x6 = x0 + 12, x7 = x0 + 14;
  f2 A = {a, a}, B = {b, b};
  for (int i = 0; i < ITERS / 2; ++i) {
    asm volatile("v_pk_fma_f32 %0, %0, %8, %9\n v_pk_fma_f32 %1, %1, %8, %9\n v_pk_fma_f32 %2, %2, %8, %9\n v_pk_fma_f32 %3, %3, %8, %9\n"
                 "v_pk_fma_f32 %4, %4, %8, %9\n v_pk_fma_f32 %5, %5, %8, %9\n v_pk_fma_f32 %6, %6, %8, %9\n v_pk_fma_f32 %7, %7, %8, %9"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(A), "v"(B));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0.x + x1.y + x2.x + x3.y + x4.x + x5.y + x6.x + x7.y;
}
template <typename K> float timeit(K k, float *d, int blocks) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1.0f, 0.5f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1.0f, 0.5f);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}
int main() {
  float *d; int blocks = 256 * 16;
  hipMalloc(&d, blocks * 256 * 4);
  float ts = timeit(k_scalar, d, blocks), tp = timeit(k_packed, d, blocks), tp8 = timeit(k_packed8, d, blocks);
  double fl = 2.0 * 8 * ITERS * (double)blocks * 256;  // FMA = 2 flop, 8 lanes-worth per iter
  printf("scalar v_fma_f32   %.3f ms  %.1f TF\n", ts, fl / ts / 1e9);
  printf("packed v_pk_fma x4 %.3f ms  %.1f TF\n", tp, fl / tp / 1e9);
  printf("packed v_pk_fma x8 %.3f ms  %.1f TF\n", tp8, fl / tp8 / 1e9);
  return 0;
}
