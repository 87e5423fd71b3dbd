// Diagnostic micro-benchmark (not part of the product): issue rate and
// SQ_INSTS_VALU accounting of packed fp32 (v_pk_fma_f32 / v_pk_add_f32)
// against scalar v_fma_f32 on gfx950.  Each kernel runs ITER iterations of
// 64 independent-ish instructions per wave; prints ms and instructions/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) (void)(x)

typedef float pf2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

__global__ __launch_bounds__(256) void k_pk_fma(float* out, float s) {
  pf2 a[8];
  for (int i = 0; i < 8; i++) a[i] = pf2{s + i, s - i};
  const pf2 m = pf2{s, s * 0.5f};
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = __builtin_elementwise_fma(a[i], m, m);
  }
  float t = 0;
  for (int i = 0; i < 8; i++) t += a[i][0] + a[i][1];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_pk_add(float* out, float s) {
  pf2 a[8];
  for (int i = 0; i < 8; i++) a[i] = pf2{s + i, s - i};
  const pf2 m = pf2{s, s * 0.5f};
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = a[i] + m;
  }
  float t = 0;
  for (int i = 0; i < 8; i++) t += a[i][0] + a[i][1];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_fma(float* out, float s) {
  float a[8];
  for (int i = 0; i < 8; i++) a[i] = s + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
  }
  float t = 0;
  for (int i = 0; i < 8; i++) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_med3(float* out, float s) {
  int a[8];
  const int lo = (int)s, hi = lo + 100;
  for (int i = 0; i < 8; i++) a[i] = lo + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int i = 0; i < 8; i++) {
        int x;
        asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(x) : "v"(a[i]), "v"(lo), "v"(hi));
        a[i] = x + 1;
      }
  }
  int t = 0;
  for (int i = 0; i < 8; i++) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = (float)t;
}

template <typename K>
void run(const char* name, K kern, float* d, int wgs) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(wgs), dim3(256), 0, 0, d, 1.0f);
  CHK(hipEventRecord(e0, 0));
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(wgs), dim3(256), 0, 0, d, 1.0f);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  const double winstr = (double)wgs * 4 * ITER * 64;  // wave instructions of the loop
  printf("%-8s %8.3f ms  %.3e wave-instr/s  (%.2f instr per SIMD-cycle at 2.4 GHz, 1024 SIMDs)\n",
         name, ms, winstr / (ms * 1e-3), winstr / (ms * 1e-3) / (1024 * 2.4e9));
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
}

int main() {
  float* d;
  const int wgs = 256 * 8;  // 8 waves' worth per SIMD... 2048 WGs of 4 waves
  CHK(hipMalloc(&d, (size_t)wgs * 256 * 4));
  run("pk_fma", k_pk_fma, d, wgs);
  run("pk_add", k_pk_add, d, wgs);
  run("fma", k_fma, d, wgs);
  run("med3", k_med3, d, wgs);
  CHK(hipFree(d));
  return 0;
}
