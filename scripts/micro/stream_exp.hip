// Micro-benchmark (not product): can a small-footprint persistent kernel
// stream a dense [B, C, r^3] fp32 grid at HBM rate, and does it leave room
// for the KNN selection beside it?  Built by scripts/micro/build_stream_exp.sh
// into scripts/micro/libstream_exp.so (ignored by git).
#include <hip/hip_runtime.h>

__global__ void stream_zero_kernel(float4* __restrict__ out, long n4, int lds_pad) {
  extern __shared__ float pad_s[];
  if (lds_pad && threadIdx.x == 0) pad_s[0] = 0.0f;
  const long stride = (long)gridDim.x * blockDim.x;
  const float4 z = {0.0f, 0.0f, 0.0f, 0.0f};
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    out[i] = z;
    out[i + stride] = z;
    out[i + 2 * stride] = z;
    out[i + 3 * stride] = z;
  }
  for (; i < n4; i += stride) out[i] = z;
}

// chunked: workgroup w owns contiguous chunks of `chunk` float4s
__global__ void stream_zero_chunk_kernel(float4* __restrict__ out, long n4, int chunk) {
  const float4 z = {0.0f, 0.0f, 0.0f, 0.0f};
  const long nchunks = (n4 + chunk - 1) / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const long base = c * chunk;
    for (int t = threadIdx.x; t < chunk; t += blockDim.x)
      if (base + t < n4) out[base + t] = z;
  }
}

// as stream_zero_kernel, with a footprint like vox_stream_kernel: `vregs`
// live VGPRs (a dependent chain the compiler cannot drop), dynamic LDS
template <int VR>
__global__ void stream_zero_fat_kernel(float4* __restrict__ out, long n4, int seed) {
  extern __shared__ float pad_s[];
  float acc[VR];
#pragma unroll
  for (int q = 0; q < VR; q++) acc[q] = (float)(seed + q + threadIdx.x);
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n4; i += stride) {
#pragma unroll
    for (int q = 0; q < VR; q++) acc[q] = acc[q] * 1.0000001f + 1.0f;
    out[i] = float4{0.0f, 0.0f, 0.0f, 0.0f};
  }
  float t = 0.0f;
#pragma unroll
  for (int q = 0; q < VR; q++) t += acc[q];
  if (t == 12345.678f) pad_s[threadIdx.x] = t;
}

extern "C" int exp_stream_fat(float* out, long n4, int wgs, int nt, int vregs, int lds_bytes,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (vregs >= 48)
    hipLaunchKernelGGL(stream_zero_fat_kernel<48>, dim3(wgs), dim3(nt), lds_bytes, st,
                       (float4*)out, n4, 1);
  else
    hipLaunchKernelGGL(stream_zero_fat_kernel<4>, dim3(wgs), dim3(nt), lds_bytes, st,
                       (float4*)out, n4, 1);
  return (int)hipGetLastError();
}

extern "C" int exp_stream(float* out, long n4, int wgs, int nt, int mode, int lds_bytes,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0)
    hipLaunchKernelGGL(stream_zero_kernel, dim3(wgs), dim3(nt), lds_bytes, st, (float4*)out, n4,
                       lds_bytes);
  else
    hipLaunchKernelGGL(stream_zero_chunk_kernel, dim3(wgs), dim3(nt), 0, st, (float4*)out, n4,
                       mode);
  return (int)hipGetLastError();
}
