// common.hpp -- shared helpers for the gfx950 kernels of libpcr_amd.so.
//
// Error convention (replaces the reference's CUDA_CHECK_ERRORS + exit(-1),
// src/cuda_utils.cuh:28-37): every C-ABI entry point returns a pcr_status and
// records a message retrievable with pcr_last_error(); the Python shim raises
// RuntimeError from it.  No entry point synchronises the device or allocates.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdarg.h>

#include "pcr_amd.h"
#include "pcr_math.h"

namespace pcr {

void set_error(const char* fmt, ...);

#define PCR_REQUIRE(cond, ...)             \
  do {                                     \
    if (!(cond)) {                         \
      ::pcr::set_error(__VA_ARGS__);       \
      return PCR_ERR_INVALID;              \
    }                                      \
  } while (0)

// Reports the launch status of the kernels just queued on `stream`.
pcr_status launch_status(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Allows a kernel to take more than the default 64 KB of dynamic LDS (gfx950
// has 160 KB per CU).  Idempotent; cheap after the first call.
template <typename K>
inline void allow_big_lds(K kernel, size_t bytes) {
  if (bytes > 48 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// knn_spatial.hip: Morton-sorted, box-pruned exact KNN.  Returns
// PCR_ERR_UNSUPPORTED without launching anything when it does not apply.
pcr_status knn_spatial(const float* xyz1, const float* xyz2, int b, int n, int m, int k,
                       float* dist1, int* idx1, float* dist2, int* idx2, const float* nrm1,
                       const float* nrm2, int relative, float* ppf1, void* ws, size_t ws_bytes,
                       bool self, hipStream_t st);

// ---------------------------------------------------------------- device
constexpr int kWave = 64;

// Inclusive block-wide scan of one int per thread (blockDim.x threads,
// multiple of 64, <= 1024).  `smem` needs blockDim.x/64 + 1 ints.
__device__ inline int block_inclusive_scan(int v, int* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int t = __shfl_up(v, off, kWave);
    if (lane >= off) v += t;
  }
  if (lane == kWave - 1) smem[wid] = v;
  __syncthreads();
  if (wid == 0) {
    int w = (lane < nw) ? smem[lane] : 0;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      int t = __shfl_up(w, off, kWave);
      if (lane >= off) w += t;
    }
    if (lane < nw) smem[lane] = w;
  }
  __syncthreads();
  int base = (wid > 0) ? smem[wid - 1] : 0;
  __syncthreads();
  return v + base;
}

__device__ inline float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ inline double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

}  // namespace pcr
