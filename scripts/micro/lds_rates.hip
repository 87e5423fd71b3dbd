// Diagnostic micro-benchmark (not product code): LDS instruction rates on
// the pattern of the KNN histogram pass.  Each variant: 512 WGs x 512
// threads (2 per CU), 4096 LDS ops per wave, cycles per op per CU reported.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(512) void k(unsigned* out, int iters, unsigned sel,
                                         const float4* __restrict__ gcand) {
  __shared__ unsigned hist[26 * 64 * 2];
  __shared__ float4 cand[256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 26 * 64 * 2; i += 512) hist[i] = 0;
  for (int i = threadIdx.x; i < 256; i += 512) cand[i] = float4{1.f * i, 2.f, 3.f, 4.f};
  __syncthreads();
  unsigned acc = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    const unsigned bin = (lane * 7 + it * 3 + wv) % 25;
    if (MODE == 0) {  // conflict-free no-return atomics, all lanes
      __hip_atomic_fetch_add(&hist[bin * 64 + lane], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 1) {  // same, 1 lane in 8 active
      if (((lane + it) & 7) == 0)
        __hip_atomic_fetch_add(&hist[bin * 64 + lane], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 2) {  // broadcast b128 reads
      const float4 v = cand[(it + wv) & 255];
      acc += __float_as_uint(v.x) ^ __float_as_uint(v.w);
    } else if (MODE == 3) {  // plain b32 stores, conflict-free
      hist[bin * 64 + lane] = it;
    } else if (MODE == 4) {  // b64 stores
      ((unsigned long long*)hist)[((bin * 64 + lane) & 1023)] = it;
    } else if (MODE == 5) {  // uniform-address vector load (buffer_load_dwordx4), L1/L2 hit
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)gcand, 0, 256 * 16, 0x00020000);
      const int off = ((it + wv) & 255) * 16;
      const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 0, off, 0));
      acc += __float_as_uint(v.x) ^ __float_as_uint(v.w);
    } else if (MODE == 7) {  // scalar load (uniform const pointer -> s_load_dwordx4)
      const float4 v = gcand[(it + wv) & 255];
      acc += __float_as_uint(v.x) ^ __float_as_uint(v.w);
    } else if (MODE == 8) {  // ds_read_b64 broadcast
      const float2 v = ((const float2*)cand)[(it + wv) & 511];
      acc += __float_as_uint(v.x) ^ __float_as_uint(v.y);
    } else if (MODE == 9) {  // ds_read_b32 broadcast
      const float v = ((const float*)cand)[(it + wv) & 1023];
      acc += __float_as_uint(v);
    } else if (MODE == 10) {  // ds_read_b128, lane-distinct consecutive addresses
      const float4 v = cand[(it + lane) & 255];
      acc += __float_as_uint(v.x) ^ __float_as_uint(v.w);
    } else if (MODE == 6) {  // three v_readlane broadcasts of per-lane registers
      const float4 v = cand[lane];
      const int t = (it + wv) & 63;
      acc += __builtin_amdgcn_readlane(__float_as_uint(v.x), t) ^ __builtin_amdgcn_readlane(__float_as_uint(v.y), t) ^ __builtin_amdgcn_readlane(__float_as_uint(v.z), t);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0);
  if (acc == sel) out[1023] = acc + hist[lane];
}

int main() {
  unsigned* d;
  hipMalloc(&d, 4096 * 4);
  unsigned h[1024];
  const int iters = 4096;
  const char* names[] = {"ds_add_u32 all lanes", "ds_add_u32 1/8 lanes", "ds_read_b128 broadcast",
                         "ds_write_b32", "ds_write_b64", "buffer_load_b128 uniform", "3x v_readlane", "s_load_dwordx4 uniform",
                         "ds_read_b64 broadcast", "ds_read_b32 broadcast", "ds_read_b128 per-lane"};
  float4* g;
  hipMalloc(&g, 256 * 16);
  hipMemset(g, 0, 256 * 16);
  for (int m = 0; m < 11; m++) {
    for (int rep = 0; rep < 2; rep++) {
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 7: hipLaunchKernelGGL(k<7>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 8: hipLaunchKernelGGL(k<8>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 9: hipLaunchKernelGGL(k<9>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
        case 10: hipLaunchKernelGGL(k<10>, dim3(512), dim3(512), 0, 0, d, iters, 7u, g); break;
      }
      hipDeviceSynchronize();
    }
    hipMemcpy(h, d, 512 * 4, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 512; i++) s += h[i];
    s /= 512;
    // 16 waves per CU (2 WGs x 8 waves), iters ops each
    printf("%-26s %8.0f cycles per WG loop -> %.2f cycles per wave-op per CU\n", names[m], s,
           s / (16.0 * iters));
  }
  return 0;
}
