// Diagnostic: checks DPP wave_ror:1 (dpp_ctrl 0x13C) on gfx950 and its cost.
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ inline float ror1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x13C, 0xF, 0xF, false));
}

__global__ __launch_bounds__(512) void check(int* out) {
  const int lane = threadIdx.x & 63;
  float v = (float)lane;
  v = ror1(v);
  out[threadIdx.x] = (int)v;
}

__global__ __launch_bounds__(512) void rate(unsigned* out, int iters) {
  const int lane = threadIdx.x & 63;
  float x = lane, y = lane * 2, z = lane * 3, acc = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      x = ror1(x);
      y = ror1(y);
      z = ror1(z);
      acc += x * y + z;
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0);
  if (acc == 12345.f) out[1000] = 1;
}

int main() {
  int* d;
  hipMalloc(&d, 4096 * 4);
  hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, d);
  int h[64];
  hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
  printf("ror1 lanes 0..5 get:");
  for (int i = 0; i < 6; i++) printf(" %d", h[i]);
  printf(" ... lane 63 gets %d\n", h[63]);
  const int iters = 4096;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(rate, dim3(512), dim3(512), 0, 0, (unsigned*)d, iters);
    hipDeviceSynchronize();
  }
  unsigned hh[512];
  hipMemcpy(hh, d, 512 * 4, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 512; i++) s += hh[i];
  s /= 512;
  // per SIMD: 4 waves; per wave 8 * iters steps of (3 dpp movs + 2 VALU)
  printf("%.0f cycles per WG -> %.2f SIMD-cycles per step (3 dpp + fma + add) per wave\n", s,
         s / (8.0 * iters) / 4.0);
  return 0;
}
