// lrf.hip -- the "change_coords" local reference frame of the reference
// model (models/pvcnn_classify.py:153-184).
//
// The reference argsorts the point norms, then walks the ranking in a Python
// loop per cloud, with a host sync per step.  Here one workgroup handles one
// cloud and needs no sort: base_x is the rank-0 point, the arg-max of
// (norm, -index).  base_y is the first qualifying point in rank order, which
// is the arg-max of the same key over the qualifying points.  So each is one
// block-wide max over 64-bit keys.  The cloud (12 B per point) is read four
// times: the mean, the two arg-max passes and the projection; 1024 threads
// per cloud, so a 65,536-point cloud is 64 points per thread per pass.
#include "common.hpp"

namespace pcr {
namespace {

constexpr int kLrfThreads = 1024;
constexpr int kLrfWaves = kLrfThreads / kWave;

__device__ inline unsigned long long block_max_u64(unsigned long long v,
                                                   unsigned long long* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = shfl_xor_u64(v, off);
    v = o > v ? o : v;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  lds_barrier();
  unsigned long long r = red[0];
#pragma unroll
  for (int w = 1; w < kLrfWaves; w++) r = red[w] > r ? red[w] : r;
  lds_barrier();  // red is reused by the next call
  return r;
}

__global__ __launch_bounds__(kLrfThreads) void lrf_kernel(const float* __restrict__ coords, int n,
                                                          float* __restrict__ new_coords,
                                                          float* __restrict__ basis_out,
                                                          int* __restrict__ picks,
                                                          int* __restrict__ status) {
  __shared__ double dred[3][kLrfWaves];
  __shared__ unsigned long long kred[kLrfWaves];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* X = coords + (size_t)b * 3 * n;

  // 1. per-axis mean in the fixed order of the voxel prep's cloud_mean (the
  //    oracle's cloud_mean_axis): thread t of 1024 sums points t, t+1024, ...
  //    ascending in double; each wave halves its 64 partials (l += l+s,
  //    s = 32..1); the 16 wave sums are halved the same way (s = 8..1).
  double s[3] = {0.0, 0.0, 0.0};
  for (int k = tid; k < n; k += kLrfThreads) {
    s[0] += (double)X[k];
    s[1] += (double)X[k + n];
    s[2] += (double)X[k + 2 * n];
  }
#pragma unroll
  for (int a = 0; a < 3; a++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_down(s[a], off, kWave);
      if (lane < off) s[a] += o;
    }
    if (lane == 0) dred[a][w] = s[a];
  }
  lds_barrier();
  float mean[3];
#pragma unroll
  for (int a = 0; a < 3; a++) {
    double v[kLrfWaves];
#pragma unroll
    for (int i = 0; i < kLrfWaves; i++) v[i] = dred[a][i];
#pragma unroll
    for (int off = kLrfWaves / 2; off > 0; off >>= 1)
#pragma unroll
      for (int i = 0; i < off; i++) v[i] += v[i + off];
    mean[a] = (float)(v[0] / (double)n);
  }

  // 2. base_x = rank 0
  unsigned long long key = 0ull;
  for (int k = tid; k < n; k += kLrfThreads) {
    const float cx = X[k] - mean[0], cy = X[k + n] - mean[1], cz = X[k + 2 * n] - mean[2];
    const unsigned long long kk = pcr_rank_key(pcr_norm3f(cx, cy, cz), k);
    key = kk > key ? kk : key;
  }
  const unsigned long long k0 = block_max_u64(key, kred);
  int st = 0, i0 = -1, i1 = -1;
  float p0[3] = {0.0f, 0.0f, 0.0f}, n0 = 0.0f, bx[3] = {0.0f, 0.0f, 0.0f};
  if (k0 == 0ull) {
    st = 1;
  } else {
    i0 = pcr_rank_key_index(k0);
    p0[0] = X[i0] - mean[0];
    p0[1] = X[i0 + n] - mean[1];
    p0[2] = X[i0 + 2 * n] - mean[2];
    n0 = pcr_norm3f(p0[0], p0[1], p0[2]);
    if (!(n0 > 1e-5f)) st = 1;  // assert base_x.norm() > 1e-5 (:159)
#pragma unroll
    for (int a = 0; a < 3; a++) bx[a] = p0[a] / n0;
  }

  // 3. base_y = the first qualifying point after rank 0 (:161-170)
  float p1[3] = {0.0f, 0.0f, 0.0f}, n1 = 0.0f;
  if (st == 0) {
    key = 0ull;
    for (int k = tid; k < n; k += kLrfThreads) {
      if (k == i0) continue;
      const float cx = X[k] - mean[0], cy = X[k + n] - mean[1], cz = X[k + 2 * n] - mean[2];
      const float nr = pcr_norm3f(cx, cy, cz);
      if (pcr_lrf_base_y_ok(cx, cy, cz, nr, bx)) {
        const unsigned long long kk = pcr_rank_key(nr, k);
        key = kk > key ? kk : key;
      }
    }
    const unsigned long long k1 = block_max_u64(key, kred);
    if (k1 == 0ull) {
      st = 2;
    } else {
      i1 = pcr_rank_key_index(k1);
      p1[0] = X[i1] - mean[0];
      p1[1] = X[i1 + n] - mean[1];
      p1[2] = X[i1 + 2 * n] - mean[2];
      n1 = pcr_norm3f(p1[0], p1[1], p1[2]);
    }
  }

  // 4. basis and projection (:174-184)
  float B[9];
#pragma unroll
  for (int a = 0; a < 9; a++) B[a] = 0.0f;
  if (st == 0) st = pcr_lrf_basis(p0, n0, p1, n1, B);
  if (st != 0) {
#pragma unroll
    for (int a = 0; a < 9; a++) B[a] = 0.0f;
  }
  float* O = new_coords + (size_t)b * 3 * n;
  for (int k = tid; k < n; k += kLrfThreads) {
    const float cx = X[k] - mean[0], cy = X[k + n] - mean[1], cz = X[k + 2 * n] - mean[2];
#pragma unroll
    for (int a = 0; a < 3; a++)
      O[k + a * n] = pcr_dot3f_nofma(B[3 * a], B[3 * a + 1], B[3 * a + 2], cx, cy, cz);
  }
  if (tid < 9) basis_out[(size_t)b * 9 + tid] = B[tid];
  if (tid == 0) {
    picks[2 * b] = i0;
    picks[2 * b + 1] = i1;
    status[b] = st;
  }
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_lrf_change_coords(const float* coords, int b, int n, float* new_coords,
                                            float* basis, int* picks, int* status, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && b <= 2147483647, "lrf_change_coords: invalid sizes b=%d n=%d",
              b, n);
  if (b == 0) return PCR_OK;
  hipLaunchKernelGGL(lrf_kernel, dim3(b), dim3(kLrfThreads), 0, as_stream(stream), coords, n,
                     new_coords, basis, picks, status);
  return launch_status("lrf_change_coords");
}
