// Diagnostic: semantics of gfx950's v_permlane16_swap / v_permlane32_swap
// with the same register as both operands (lane values after the swap).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned a = threadIdx.x, b = threadIdx.x;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0\n\ts_nop 1" : "+v"(a));
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0\n\ts_nop 1" : "+v"(b));
  o[threadIdx.x] = a;
  o[64 + threadIdx.x] = b;
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("permlane16_swap(a,a):");
  for (int i = 0; i < 64; i++) printf(" %u", h[i]);
  printf("\npermlane32_swap(a,a):");
  for (int i = 0; i < 64; i++) printf(" %u", h[64 + i]);
  printf("\n");
  return 0;
}
