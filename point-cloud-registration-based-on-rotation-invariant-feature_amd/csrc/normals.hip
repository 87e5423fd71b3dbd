// normals.hip -- point normals by radius-neighbourhood PCA (SURVEY.md 8f row
// f3).  This is the Open3D call the reference makes on the host for every
// registration sample (utils/open3d_func.py:77-83: estimate_normals with
// KDTreeSearchParamRadius(0.1), orient_normals_towards_camera_location(),
// normalize_normals(); called from datasets/deepgmr_mn40.py).  Open3D is
// absent here: the per-point arithmetic is the restatement in
// include/pcr_math.h (pcr_estimate_normal), and parity against Open3D is
// unpinned.
//
// Layout: one workgroup takes 256 query points of one cloud.  The cloud
// streams through LDS in 2048-point tiles (24 KB).  Every thread scans each
// tile in ascending index order and keeps its nine fp64 cumulants in
// registers.  The radius test is in double, as Open3D (double points) does
// it: |q - p|^2 < radius^2.  For the c2 clouds (1024 points) that is about
// 1M candidate tests per cloud, and the stage is fp64-VALU bound at a few
// microseconds per batch.
#include "common.hpp"

namespace pcr {
namespace {

constexpr int kNrmThreads = 256;
constexpr int kNrmTile = 2048;

__global__ __launch_bounds__(kNrmThreads) void normals_kernel(const float* __restrict__ pts, int n,
                                                              double r2,
                                                              float* __restrict__ normals,
                                                              int* __restrict__ counts) {
  __shared__ __align__(16) float tile[3][kNrmTile];
  const float r2f_hi = (float)(r2 * 1.0001) * 1.0001f;
  const int b = blockIdx.y;
  const int j = blockIdx.x * kNrmThreads + threadIdx.x;
  const bool active = j < n;
  const float* P = pts + (size_t)b * 3 * n;
  float qx = 0.0f, qy = 0.0f, qz = 0.0f;
  if (active) {
    qx = P[j];
    qy = P[j + n];
    qz = P[j + 2 * n];
  }
  const double dqx = qx, dqy = qy, dqz = qz;
  double cum[9];
#pragma unroll
  for (int a = 0; a < 9; a++) cum[a] = 0.0;
  int cnt = 0;
  for (int t0 = 0; t0 < n; t0 += kNrmTile) {
    const int tc = min(kNrmTile, n - t0);
    __syncthreads();
    for (int q = threadIdx.x; q < tc; q += kNrmThreads) {
      tile[0][q] = P[t0 + q];
      tile[1][q] = P[t0 + q + n];
      tile[2][q] = P[t0 + q + 2 * n];
    }
    __syncthreads();
    if (active) {
      // fp32 prefilter (float4 reads, four candidates per test): the fp32
      // distance is within ~3e-7 relative of the exact one, so a candidate
      // above r2f_hi cannot pass the fp64 test, which alone decides
      auto take = [&](float xf, float yf, float zf) {
        const double x = xf, y = yf, z = zf;
        const double dx = dqx - x, dy = dqy - y, dz = dqz - z;
        const double d2 = (dx * dx + dy * dy) + dz * dz;
        if (d2 < r2) {
          cum[0] += x;
          cum[1] += y;
          cum[2] += z;
          cum[3] += x * x;
          cum[4] += x * y;
          cum[5] += x * z;
          cum[6] += y * y;
          cum[7] += y * z;
          cum[8] += z * z;
          cnt++;
        }
      };
      const int t4 = tc & ~3;
      for (int q = 0; q < t4; q += 4) {
        const float4 X = *reinterpret_cast<const float4*>(&tile[0][q]);
        const float4 Y = *reinterpret_cast<const float4*>(&tile[1][q]);
        const float4 Z = *reinterpret_cast<const float4*>(&tile[2][q]);
        const float xs[4] = {X.x, X.y, X.z, X.w}, ys[4] = {Y.x, Y.y, Y.z, Y.w},
                    zs[4] = {Z.x, Z.y, Z.z, Z.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const float ex = qx - xs[u], ey = qy - ys[u], ez = qz - zs[u];
          if (pcr_sumsq3f_nofma(ex, ey, ez) <= r2f_hi) take(xs[u], ys[u], zs[u]);
        }
      }
      for (int q = t4; q < tc; q++) take(tile[0][q], tile[1][q], tile[2][q]);
    }
  }
  if (!active) return;
  float nv[3];
  pcr_estimate_normal(cum, cnt, qx, qy, qz, nv);
  float* N = normals + (size_t)b * 3 * n;
  N[j] = nv[0];
  N[j + n] = nv[1];
  N[j + 2 * n] = nv[2];
  if (counts) counts[(size_t)b * n + j] = cnt;
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_estimate_normals(const float* points, int b, int n, double radius,
                                           float* normals, int* counts, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 0 && b <= 65535, "estimate_normals: invalid sizes b=%d n=%d", b, n);
  PCR_REQUIRE(radius > 0.0, "estimate_normals: radius must be positive");
  if (b == 0 || n == 0) return PCR_OK;
  hipLaunchKernelGGL(normals_kernel, dim3(ceil_div(n, kNrmThreads), b), dim3(kNrmThreads), 0,
                     as_stream(stream), points, n, radius * radius, normals, counts);
  return launch_status("estimate_normals");
}
