// pointnet2.hip -- the PointNet++ ops of the reference extension (SURVEY.md
// 8f row f4): gather_features fwd/bwd and furthest_point_sampling
// (src/sampling/sampling.cu:18-173), three_nearest_neighbors_interpolate
// fwd/bwd (src/interpolate/neighbor_interpolate.cu:21-171).
//
// MI355X layout choices:
//  - FPS keeps a cloud's coordinates and point-to-set distances in registers
//    (clouds <= 8192 points, 256 threads).  Each sample step needs one barrier:
//    every wave posts its best (key, xyz) to an LDS slot, and the slots
//    alternate between steps.  The reference does a 9-level LDS tree with a
//    barrier per level, and re-reads the chosen point from global memory.
//    Bigger clouds keep the distances in a workspace and stream the points.
//  - three-NN stages the centres in LDS tiles.  One thread owns one point,
//    and the interpolation is fused into the same kernel: the indices and
//    weights never round-trip through HBM before they are used.
#include "common.hpp"

namespace pcr {
namespace {

// ------------------------------------------------------------------ gather
__global__ __launch_bounds__(256) void gather_fwd_kernel(const float* __restrict__ feat,
                                                          const int* __restrict__ idx, int c,
                                                          int n, int m, int64_t total,
                                                          float* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * 256) {
    const int j = (int)(t % m);
    const int64_t bc = t / m;
    const int b = (int)(bc / c);
    const int i = idx[(int64_t)b * m + j];
    out[t] = (i >= 0 && i < n) ? feat[bc * n + i] : 0.0f;
  }
}

__global__ __launch_bounds__(256) void gather_bwd_kernel(const float* __restrict__ gy,
                                                          const int* __restrict__ idx, int c,
                                                          int n, int m, int64_t total,
                                                          float* __restrict__ gx) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * 256) {
    const int j = (int)(t % m);
    const int64_t bc = t / m;
    const int b = (int)(bc / c);
    const int i = idx[(int64_t)b * m + j];
    if (i >= 0 && i < n) atomicAdd(gx + bc * n + i, gy[t]);
  }
}

// --------------------------------------------------------------------- FPS
constexpr int kFpsThreads = 256;
constexpr int kFpsWaves = kFpsThreads / kWave;
constexpr int kFpsMaxE = 32;  // register path: n <= 8192

struct FpsSlot {
  unsigned long long key;
  float x, y, z, pad;
};

__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = shfl_xor_u64(v, off);
    v = o > v ? o : v;
  }
  return v;
}

// Posts this wave's best (key, xyz) and returns the workgroup's best after
// the single barrier.  slots[2][NWV]; parity alternates per step, so a slot
// is rewritten only after every wave has passed the next barrier.
template <int NWV = kFpsWaves>
__device__ inline FpsSlot fps_block_best(unsigned long long key, float x, float y, float z,
                                         FpsSlot (*slots)[NWV], int parity) {
  const unsigned long long wbest = wave_max_u64(key);
  if (key == wbest && wbest != 0ull) {  // keys are unique: exactly one lane
    FpsSlot s;
    s.key = wbest;
    s.x = x;
    s.y = y;
    s.z = z;
    s.pad = 0.0f;
    slots[parity][threadIdx.x >> 6] = s;
  } else if (wbest == 0ull && (threadIdx.x & 63) == 0) {
    slots[parity][threadIdx.x >> 6].key = 0ull;
  }
  lds_barrier();
  FpsSlot best = slots[parity][0];
#pragma unroll
  for (int w = 1; w < NWV; w++) {
    const FpsSlot s = slots[parity][w];
    if (s.key > best.key) best = s;
  }
  return best;
}

template <int E>
__global__ __launch_bounds__(kFpsThreads) void fps_reg_kernel(const float* __restrict__ coords,
                                                                int n, int m,
                                                                int* __restrict__ indices) {
  __shared__ FpsSlot slots[2][kFpsWaves];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* xs = coords + (size_t)b * 3 * n;
  int* out = indices + (size_t)b * m;
  float px[E], py[E], pz[E], dist[E];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int k = e * kFpsThreads + tid;
    const bool ok = k < n;
    px[e] = ok ? xs[k] : 0.0f;
    py[e] = ok ? xs[k + n] : 0.0f;
    pz[e] = ok ? xs[k + 2 * n] : 0.0f;
    dist[e] = 1e38f;  // sampling.cpp:52 torch::full(1e38f)
  }
  // the first sample is point 0 (sampling.cu:104-106)
  float x1 = xs[0], y1 = xs[n], z1 = xs[2 * n];
  if (tid == 0) out[0] = 0;
  for (int j = 1; j < m; j++) {
    unsigned long long key = 0ull;
    float bx = 0.0f, by = 0.0f, bz = 0.0f;
#pragma unroll
    for (int e = 0; e < E; e++) {
      const int k = e * kFpsThreads + tid;
      if (k < n) {
        const float d = pcr_sumsq3f(px[e] - x1, py[e] - y1, pz[e] - z1);
        dist[e] = fminf(d, dist[e]);
        const unsigned long long kk = pcr_fps_key(dist[e], k);
        if (kk > key) {
          key = kk;
          bx = px[e];
          by = py[e];
          bz = pz[e];
        }
      }
    }
    const FpsSlot best = fps_block_best(key, bx, by, bz, slots, j & 1);
    x1 = best.x;
    y1 = best.y;
    z1 = best.z;
    if (tid == 0) out[j] = pcr_fps_key_index(best.key);
  }
}

// clouds beyond the register path: distances in the workspace, points
// streamed from global memory (L2-resident) every step; 1024 threads, so a
// thread walks n / 1024 points per step
constexpr int kFpsBigThreads = 1024;
__global__ __launch_bounds__(kFpsBigThreads) void fps_big_kernel(const float* __restrict__ coords,
                                                                  int n, int m,
                                                                  float* __restrict__ dist_ws,
                                                                  int* __restrict__ indices) {
  constexpr int NWV = kFpsBigThreads / kWave;
  __shared__ FpsSlot slots[2][NWV];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* xs = coords + (size_t)b * 3 * n;
  float* dist = dist_ws + (size_t)b * n;
  int* out = indices + (size_t)b * m;
  for (int k = tid; k < n; k += kFpsBigThreads) dist[k] = 1e38f;
  float x1 = xs[0], y1 = xs[n], z1 = xs[2 * n];
  if (tid == 0) out[0] = 0;
  for (int j = 1; j < m; j++) {
    unsigned long long key = 0ull;
    float bx = 0.0f, by = 0.0f, bz = 0.0f;
    for (int k = tid; k < n; k += kFpsBigThreads) {
      const float x = xs[k], y = xs[k + n], z = xs[k + 2 * n];
      const float dd = fminf(pcr_sumsq3f(x - x1, y - y1, z - z1), dist[k]);
      dist[k] = dd;  // each thread owns its points: no cross-thread hazard
      const unsigned long long kk = pcr_fps_key(dd, k);
      if (kk > key) {
        key = kk;
        bx = x;
        by = y;
        bz = z;
      }
    }
    const FpsSlot best = fps_block_best<NWV>(key, bx, by, bz, slots, j & 1);
    x1 = best.x;
    y1 = best.y;
    z1 = best.z;
    if (tid == 0) out[j] = pcr_fps_key_index(best.key);
  }
}

// ---------------------------------------------------------- three NN
constexpr int kNnThreads = 256;
constexpr int kNnTile = 1024;  // centres per LDS tile (12 KB)

__global__ __launch_bounds__(kNnThreads) void three_nn_kernel(
    const float* __restrict__ points, const float* __restrict__ centers,
    const float* __restrict__ cfeat, int c, int m, int n, float* __restrict__ out,
    int* __restrict__ inds, float* __restrict__ wgts) {
  __shared__ __align__(16) float tile[3][kNnTile];
  const int b = blockIdx.y;
  const int j = blockIdx.x * kNnThreads + threadIdx.x;
  const bool active = j < n;
  const float* P = points + (size_t)b * 3 * n;
  const float* C = centers + (size_t)b * 3 * m;
  float ux = 0.0f, uy = 0.0f, uz = 0.0f;
  if (active) {
    ux = P[j];
    uy = P[j + n];
    uz = P[j + 2 * n];
  }
  float best[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  int besti[3] = {0, 0, 0};
  for (int t0 = 0; t0 < m; t0 += kNnTile) {
    const int cnt = min(kNnTile, m - t0);
    __syncthreads();
    for (int q = threadIdx.x; q < cnt; q += kNnThreads) {
      tile[0][q] = C[t0 + q];
      tile[1][q] = C[t0 + q + m];
      tile[2][q] = C[t0 + q + 2 * m];
    }
    __syncthreads();
    if (active) {
      // four candidates per broadcast ds_read_b128 of x, y and z; the
      // distances are computed before the (rarely taken) insertions, which
      // stay in candidate order
      const int c4 = cnt & ~3;
      for (int q = 0; q < c4; q += 4) {
        const float4 X = *reinterpret_cast<const float4*>(&tile[0][q]);
        const float4 Y = *reinterpret_cast<const float4*>(&tile[1][q]);
        const float4 Z = *reinterpret_cast<const float4*>(&tile[2][q]);
        // (ux - x)^2 + (uy - y)^2 + (uz - z)^2 (neighbor_interpolate.cu:42)
        const float d0 = pcr_sumsq3f(ux - X.x, uy - Y.x, uz - Z.x);
        const float d1 = pcr_sumsq3f(ux - X.y, uy - Y.y, uz - Z.y);
        const float d2 = pcr_sumsq3f(ux - X.z, uy - Y.z, uz - Z.z);
        const float d3 = pcr_sumsq3f(ux - X.w, uy - Y.w, uz - Z.w);
        if (fminf(fminf(d0, d1), fminf(d2, d3)) < best[2]) {
          pcr_three_nn_insert(d0, t0 + q, best, besti);
          pcr_three_nn_insert(d1, t0 + q + 1, best, besti);
          pcr_three_nn_insert(d2, t0 + q + 2, best, besti);
          pcr_three_nn_insert(d3, t0 + q + 3, best, besti);
        }
      }
      for (int q = c4; q < cnt; q++) {
        const float d = pcr_sumsq3f(ux - tile[0][q], uy - tile[1][q], uz - tile[2][q]);
        pcr_three_nn_insert(d, t0 + q, best, besti);
      }
    }
  }
  if (!active) return;
  float w[3];
  pcr_three_nn_weights(best, w);
  if (blockIdx.z == 0) {
    float* W = wgts + (size_t)b * 3 * n;
    int* I = inds + (size_t)b * 3 * n;
#pragma unroll
    for (int a = 0; a < 3; a++) {
      W[j + a * n] = w[a];
      I[j + a * n] = besti[a];
    }
  }
  // channel group blockIdx.z: the (cheap) scan is repeated per group so the
  // gathers of the interpolation spread over gridDim.z times more waves
  const int cpg = (c + gridDim.z - 1) / gridDim.z;
  const int ch0 = blockIdx.z * cpg, ch1 = min(c, ch0 + cpg);
  const float* F = cfeat + (size_t)b * c * m;
  float* O = out + (size_t)b * c * n;
#pragma unroll 4
  for (int ch = ch0; ch < ch1; ch++) {
    const float* f = F + (size_t)ch * m;
    // no centres at all: the reference reads feature 0 of an empty tensor
    O[(size_t)ch * n + j] =
        m > 0 ? pcr_wsum3(f[besti[0]], w[0], f[besti[1]], w[1], f[besti[2]], w[2]) : 0.0f;
  }
}

__global__ __launch_bounds__(256) void three_nn_grad_kernel(const float* __restrict__ gy,
                                                             const int* __restrict__ inds,
                                                             const float* __restrict__ wgts,
                                                             int c, int n, int m, int64_t total,
                                                             float* __restrict__ gx) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * 256) {
    const int j = (int)(t % n);
    const int64_t bc = t / n;
    const int b = (int)(bc / c);
    const float g = gy[t];
    const int* I = inds + (size_t)b * 3 * n;
    const float* W = wgts + (size_t)b * 3 * n;
    float* G = gx + bc * m;
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const int i = I[j + a * n];
      if (i >= 0 && i < m) atomicAdd(G + i, W[j + a * n] * g);
    }
  }
}

inline unsigned grid_for(int64_t total) {
  const int64_t blocks = ceil_div64(total, 256);
  return (unsigned)(blocks < 65536 ? (blocks > 0 ? blocks : 1) : 65536);
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_gather_features_forward(const float* features, const int* indices,
                                                  int b, int c, int n, int m, float* out,
                                                  void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 1 && m >= 0, "gather_features_forward: invalid sizes");
  const int64_t total = (int64_t)b * c * m;
  if (total == 0) return PCR_OK;
  hipLaunchKernelGGL(gather_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                     features, indices, c, n, m, total, out);
  return launch_status("gather_features_forward");
}

extern "C" pcr_status pcr_gather_features_backward(const float* grad_y, const int* indices,
                                                   int b, int c, int n, int m, float* grad_x,
                                                   void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && m >= 0, "gather_features_backward: invalid sizes");
  const int64_t gx_elems = (int64_t)b * c * n;
  if (gx_elems == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(grad_x, 0, (size_t)gx_elems * 4, st) != hipSuccess)
    return launch_status("gather_features_backward memset");
  const int64_t total = (int64_t)b * c * m;
  if (total > 0)
    hipLaunchKernelGGL(gather_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, grad_y,
                       indices, c, n, m, total, grad_x);
  return launch_status("gather_features_backward");
}

extern "C" size_t pcr_fps_workspace_size(int b, int n) {
  if (b <= 0 || n <= kFpsThreads * kFpsMaxE) return 256;
  return (size_t)b * n * 4;
}

extern "C" pcr_status pcr_furthest_point_sampling(const float* coords, int b, int n, int m,
                                                  int* indices, void* workspace,
                                                  size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && m >= 0, "furthest_point_sampling: invalid sizes b=%d n=%d m=%d",
              b, n, m);
  PCR_REQUIRE(b <= 2147483647 / 3 && (int64_t)n * 3 < 2147483647,
              "furthest_point_sampling: cloud too large");
  if (b == 0 || m == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  const dim3 grid(b), block(kFpsThreads);
  const int e = ceil_div(n, kFpsThreads);
  if (e <= 1)
    hipLaunchKernelGGL(fps_reg_kernel<1>, grid, block, 0, st, coords, n, m, indices);
  else if (e <= 2)
    hipLaunchKernelGGL(fps_reg_kernel<2>, grid, block, 0, st, coords, n, m, indices);
  else if (e <= 4)
    hipLaunchKernelGGL(fps_reg_kernel<4>, grid, block, 0, st, coords, n, m, indices);
  else if (e <= 8)
    hipLaunchKernelGGL(fps_reg_kernel<8>, grid, block, 0, st, coords, n, m, indices);
  else if (e <= 16)
    hipLaunchKernelGGL(fps_reg_kernel<16>, grid, block, 0, st, coords, n, m, indices);
  else if (e <= kFpsMaxE)
    hipLaunchKernelGGL(fps_reg_kernel<kFpsMaxE>, grid, block, 0, st, coords, n, m, indices);
  else {
    const size_t need = pcr_fps_workspace_size(b, n);
    PCR_REQUIRE(workspace != nullptr && workspace_bytes >= need,
                "furthest_point_sampling: workspace too small (%zu < %zu)", workspace_bytes, need);
    hipLaunchKernelGGL(fps_big_kernel, grid, dim3(kFpsBigThreads), 0, st, coords, n, m,
                       (float*)workspace, indices);
  }
  return launch_status("furthest_point_sampling");
}

extern "C" pcr_status pcr_three_nn_interpolate_forward(const float* points, const float* centers,
                                                       const float* centers_features, int b,
                                                       int c, int m, int n, float* out,
                                                       int* indices, float* weights,
                                                       void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && m >= 0 && n >= 0 && b <= 65535,
              "three_nearest_neighbors_interpolate_forward: invalid sizes");
  if (b == 0 || n == 0) return PCR_OK;
  const int cgroups = c >= 64 ? 4 : (c >= 16 ? 2 : 1);
  hipLaunchKernelGGL(three_nn_kernel, dim3(ceil_div(n, kNnThreads), b, cgroups), dim3(kNnThreads), 0,
                     as_stream(stream), points, centers, centers_features, c, m, n, out, indices,
                     weights);
  return launch_status("three_nearest_neighbors_interpolate_forward");
}

extern "C" pcr_status pcr_three_nn_interpolate_backward(const float* grad_y, const int* indices,
                                                        const float* weights, int b, int c, int n,
                                                        int m, float* grad_x, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && m >= 0,
              "three_nearest_neighbors_interpolate_backward: invalid sizes");
  const int64_t gx_elems = (int64_t)b * c * m;
  if (gx_elems == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(grad_x, 0, (size_t)gx_elems * 4, st) != hipSuccess)
    return launch_status("three_nearest_neighbors_interpolate_backward memset");
  const int64_t total = (int64_t)b * c * n;
  if (total > 0)
    hipLaunchKernelGGL(three_nn_grad_kernel, dim3(grid_for(total)), dim3(256), 0, st, grad_y,
                       indices, weights, c, n, m, total, grad_x);
  return launch_status("three_nearest_neighbors_interpolate_backward");
}
