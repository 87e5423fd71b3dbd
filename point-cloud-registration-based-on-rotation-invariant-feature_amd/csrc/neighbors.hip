// neighbors.hip -- neighbour search (KNN, ball query), grouping, point-pair
// features (global and local) and the math self-test hooks, for gfx950.
//
// Replaces (relative to the reference's PVCNN/modules/functional/src):
//   knn/knn.cu:5-98               KnnKernel / KnnGradKernel
//   spherical_ppf/ppf.cu:19-99    spherical_ppf_kernel
//   ball_query/ball_query.cu:19-59
//   grouping/grouping.cu:18-85
// and the PyTorch local-PPF block of PVCNN/models/pvcnn_classify.py:252-269.
//
// KNN: the reference keeps each query's top-k in GLOBAL memory and runs an
// O(k) bubble pass per candidate with one workgroup per cloud.  Here each
// thread owns one query and keeps its top-k in registers (a compile-time
// sized, statically indexed sorted array, branch-free insertion), the
// candidate cloud is staged through LDS in coalesced tiles shared by the
// 256 queries of the workgroup, and the grid spans (query blocks x clouds).
// Candidates are scanned in ascending index with a strict `<` test, which is
// exactly the reference's tie rule (lower index first); slots that never fill
// keep (10000, 0) as the reference's ones*10000 / zeros init.
#include "common.hpp"

namespace pcr {

constexpr int kKnnThreads = 256;
constexpr int kKnnTile = 1024;
constexpr int kMaxC = 8;

// Sorted ascending; valid region is the LAST k slots, the first KMAX-k slots
// hold -inf and are never displaced.  Insert (d, j) if d < D[KMAX-1].
template <int KMAX>
struct TopK {
  float d[KMAX];
  int j[KMAX];
  __device__ void init(int k) {
#pragma unroll
    for (int q = 0; q < KMAX; q++) {
      d[q] = (q < KMAX - k) ? -__builtin_inff() : PCR_KNN_UNDEF;
      j[q] = 0;
    }
  }
  __device__ float thr() const { return d[KMAX - 1]; }
  // Insertion as a compare-exchange carry chain: the new element passes every
  // slot it is not strictly smaller than (equal distances keep the earlier,
  // lower index first); from its slot on, every element shifts by one
  // (`ins`), so equal displaced elements keep their order.  A non-qualifying
  // x (>= D[KMAX-1], or NaN) falls off the end unchanged.  Lane masks are
  // short-lived (no SGPR pressure, unlike a hoisted compare-all form).
  __device__ void insert(float x, int jx) {
    bool ins = false;
#pragma unroll
    for (int q = 0; q < KMAX; q++) {
      const bool lt = ins || (x < d[q]);
      const float nd = lt ? x : d[q];
      const int nj = lt ? jx : j[q];
      x = lt ? d[q] : x;
      jx = lt ? j[q] : jx;
      d[q] = nd;
      j[q] = nj;
      ins = lt;
    }
  }
};

// Distance with the reference's contraction: d = t0*t0, d = fma(tp, tp, d)
// (knn.cu:20-24 under nvcc --fmad=true).
template <int KMAX, bool PPF, int CC>
__global__ __launch_bounds__(kKnnThreads) void knn_kernel(
    const float* __restrict__ xyz1, const float* __restrict__ xyz2, int c, int n, int m, int k,
    float* __restrict__ dist, int* __restrict__ idx,
    // fused local PPF (self KNN): normals of xyz1 (== xyz2), output [b,4,k,n]
    const float* __restrict__ normals, int relative, float* __restrict__ ppf) {
  __shared__ float tile_s[kMaxC * kKnnTile];
  const int b = blockIdx.y;
  const int i = blockIdx.x * kKnnThreads + threadIdx.x;
  const bool active = i < n;
  const float* x1 = xyz1 + (size_t)b * c * n;
  const float* x2 = xyz2 + (size_t)b * c * m;
  // CC == 3: the xyz specialisation; CC == kMaxC: generic c <= kMaxC
  float q[CC];
#pragma unroll
  for (int p = 0; p < CC; p++) q[p] = (p < c && active) ? x1[i + (size_t)p * n] : 0.0f;
  TopK<KMAX> top;
  top.init(k);
  for (int t0 = 0; t0 < m; t0 += kKnnTile) {
    const int tl = min(kKnnTile, m - t0);
    __syncthreads();
    for (int p = 0; p < c; p++)
      for (int t = threadIdx.x; t < tl; t += kKnnThreads)
        tile_s[p * kKnnTile + t] = x2[(size_t)p * m + t0 + t];
    __syncthreads();
    if (active) {
      if (CC == 3) {
#pragma unroll 1
        for (int t = 0; t < tl; t++) {
          const float a = q[0] - tile_s[t];
          const float bb = q[1] - tile_s[kKnnTile + t];
          const float cc = q[2] - tile_s[2 * kKnnTile + t];
          float d = a * a;
          d = __builtin_fmaf(bb, bb, d);
          d = __builtin_fmaf(cc, cc, d);
          if (__any(d < top.thr())) top.insert(d, t0 + t);  // no-op for d >= thr
        }
      } else {
#pragma unroll 1
        for (int t = 0; t < tl; t++) {
          float d = 0.0f;
#pragma unroll
          for (int p = 0; p < CC; p++) {
            if (p < c) {
              const float a = q[p] - tile_s[p * kKnnTile + t];
              d = (p == 0) ? a * a : __builtin_fmaf(a, a, d);
            }
          }
          if (__any(d < top.thr())) top.insert(d, t0 + t);  // no-op for d >= thr
        }
      }
    }
  }
  if (!active) return;
  const int base = KMAX - k;
#pragma unroll
  for (int s = 0; s < KMAX; s++) {
    if (s >= base) {
      const size_t o = ((size_t)b * k + (s - base)) * n + i;
      if (dist) dist[o] = top.d[s];
      if (idx) idx[o] = top.j[s];
    }
  }
  if (PPF) {
    // neighbour ids re-read from the rows this thread just wrote (idx is
    // required for the fused variant) to keep the slot loop rolled
    const float* nb = normals + (size_t)b * 3 * n;
    const float cnx = nb[i], cny = nb[i + n], cnz = nb[i + 2 * n];
#pragma unroll 1
    for (int slot = 0; slot < k; slot++) {
      const int jn = idx[((size_t)b * k + slot) * n + i];
      float o[4];
      pcr_local_ppf(q[0], q[1], q[2], cnx, cny, cnz, x2[jn], x2[jn + m], x2[jn + 2 * m], nb[jn],
                    nb[jn + n], nb[jn + 2 * n], relative, o);
#pragma unroll
      for (int ch = 0; ch < 4; ch++) ppf[(((size_t)b * 4 + ch) * k + slot) * n + i] = o[ch];
    }
  }
}

// k > 128: the reference algorithm itself (top-k in the output buffers).
__global__ __launch_bounds__(256) void knn_generic_kernel(const float* __restrict__ xyz1,
                                                          const float* __restrict__ xyz2, int c,
                                                          int n, int m, int k,
                                                          float* __restrict__ dist,
                                                          int* __restrict__ idx) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* x1 = xyz1 + (size_t)b * c * n;
  const float* x2 = xyz2 + (size_t)b * c * m;
  float* D = dist + (size_t)b * k * n;
  int* I = idx + (size_t)b * k * n;
  for (int q = 0; q < k; q++) {
    D[i + (size_t)q * n] = PCR_KNN_UNDEF;
    I[i + (size_t)q * n] = 0;
  }
  for (int j = 0; j < m; j++) {
    float d = 0.0f;
    for (int p = 0; p < c; p++) {
      const float a = x1[i + (size_t)p * n] - x2[j + (size_t)p * m];
      d = (p == 0) ? a * a : __builtin_fmaf(a, a, d);
    }
    if (d < D[i + (size_t)(k - 1) * n]) {
      int q = k - 1;
      while (q > 0 && d < D[i + (size_t)(q - 1) * n]) {
        D[i + (size_t)q * n] = D[i + (size_t)(q - 1) * n];
        I[i + (size_t)q * n] = I[i + (size_t)(q - 1) * n];
        q--;
      }
      D[i + (size_t)q * n] = d;
      I[i + (size_t)q * n] = j;
    }
  }
}

// knn.cu:52-78: one direction, atomically accumulated into both grads.
__global__ __launch_bounds__(256) void knn_grad_kernel(const float* __restrict__ x1,
                                                       const float* __restrict__ x2, int c, int n,
                                                       int m, int k, const float* __restrict__ gd,
                                                       const int* __restrict__ id,
                                                       float* __restrict__ g1,
                                                       float* __restrict__ g2) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x1 += (size_t)b * c * n;
  x2 += (size_t)b * c * m;
  gd += (size_t)b * k * n;
  id += (size_t)b * k * n;
  g1 += (size_t)b * c * n;
  g2 += (size_t)b * c * m;
  for (int q = 0; q < k; q++) {
    const float g = gd[i + (size_t)q * n] * 2.0f;
    if (g >= 20000.0f) continue;
    const int j = id[i + (size_t)q * n];
    if (j < 0 || j >= m) continue;
    for (int p = 0; p < c; p++) {
      const float t = g * (x1[i + (size_t)p * n] - x2[j + (size_t)p * m]);
      atomicAdd(g1 + i + (size_t)p * n, t);
      atomicAdd(g2 + j + (size_t)p * m, -t);
    }
  }
}

// KNN backward without atomics (contract knn.cu:52-78, both launches of
// knn.cu:88-98): every output element is a gather of its own terms in a
// fixed order, so the gradient is bit-repeatable.  Point i of cloud A gets
//   sum_q  g(q,i) (xA[i] - xB[idxA(q,i)])                    own slots
//   - sum over the pairs (q, i') of cloud B's direction with idxB(q,i') = i
//         of g(q,i') (xB[i'] - xA[i])                         as a neighbour
// with g = 2 graddist skipped at >= 20000, every term the reference's own
// product.  The second sum needs, per target point, the list of pairs that
// name it: knn_bwd_sort_kernel counts each direction's pairs per target (one
// workgroup per (cloud, direction), LDS counters: the segment starts) and
// orders them by target, ascending pair id within a target, with a stable
// workgroup radix sort (O(P) per pass), and knn_bwd_gather_kernel sums, one
// thread per point.
constexpr int kKnnBwdThreads = 1024;
constexpr int kKnnBwdMaxT = 16384;  // targets per cloud the LDS counters hold

struct KnnBwdWs {
  int* start[2];  // [b][T_d + 1] segment starts of direction d (by target)
  int* list[2];   // [b][k N_d] pair ids (q N_d + i) by target, ascending within a target
  int* tmp[2];    // [b][k N_d] the radix sort's second buffer
};

static size_t knn_bwd_ws_layout(int b, int n, int m, int k, KnnBwdWs* w, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off = (off + bytes + 255) / 256 * 256;
    return (int*)q;
  };
  const int N[2] = {n, m}, T[2] = {m, n};
  for (int d = 0; d < 2; d++) {
    int* s = take((size_t)b * (T[d] + 1) * 4);
    int* l = take((size_t)b * k * N[d] * 4);
    int* t = take((size_t)b * k * N[d] * 4);
    if (w) {
      w->start[d] = s;
      w->list[d] = l;
      w->tmp[d] = t;
    }
  }
  return off;
}

__global__ __launch_bounds__(kKnnBwdThreads) void knn_bwd_sort_kernel(
    const float* __restrict__ gd0, const int* __restrict__ idx0, const float* __restrict__ gd1,
    const int* __restrict__ idx1, int n, int m, int k, KnnBwdWs ws) {
  extern __shared__ int cnt_s[];  // [T]
  __shared__ int scan_s[kKnnBwdThreads / kWave + 1];
  __shared__ int rs_lds[(2 + kKnnBwdThreads / kWave) * 256];  // wg_radix_sort
  const int b = blockIdx.x, d = blockIdx.y, tid = threadIdx.x;
  const int N = d ? m : n, T = d ? n : m;
  const size_t P = (size_t)k * N;
  const float* gd = (d ? gd1 : gd0) + (size_t)b * P;
  const int* idx = (d ? idx1 : idx0) + (size_t)b * P;
  int* start = ws.start[d] + (size_t)b * (T + 1);
  int* list = ws.list[d] + (size_t)b * P;
  int* tmp = ws.tmp[d] + (size_t)b * P;
  auto target = [&](size_t p) {
    const float g = gd[p] * 2.0f;
    const int j = idx[p];
    return (!(g >= 20000.0f) && j >= 0 && j < T) ? j : -1;  // knn.cu:68: NaN is not skipped
  };
  for (int t = tid; t < T; t += kKnnBwdThreads) cnt_s[t] = 0;
  __syncthreads();
  for (size_t p = tid; p < P; p += kKnnBwdThreads) {
    const int j = target(p);
    if (j >= 0) atomicAdd(&cnt_s[j], 1);
  }
  __syncthreads();
  {
    const int chunk = (T + kKnnBwdThreads - 1) / kKnnBwdThreads;
    const int t0 = min(T, tid * chunk), t1 = min(T, t0 + chunk);
    int sum = 0;
    for (int t = t0; t < t1; t++) sum += cnt_s[t];
    const int incl = block_inclusive_scan(sum, scan_s);
    int run = incl - sum;
    for (int t = t0; t < t1; t++) {
      const int c = cnt_s[t];
      start[t] = run;
      run += c;
    }
    if (tid == kKnnBwdThreads - 1) start[T] = incl;
  }
  __syncthreads();
  // the pairs by target, ascending pair id within a target: a stable LSD
  // radix sort of the pair ids keyed by target (invalid pairs key T: last).
  // O(P) per pass, whatever the targets' multiplicities (a hub neighbour
  // named by thousands of pairs costs no more than any other target)
  for (size_t p = tid; p < P; p += kKnnBwdThreads) list[p] = (int)p;
  __threadfence_block();
  __syncthreads();
  const int kbits = 32 - __clz(T);  // keys 0 .. T
  int* res = wg_radix_sort<kKnnBwdThreads>(
      list, tmp, (int)P, kbits,
      [&](int p) {
        const int j = target((size_t)p);
        return j >= 0 ? j : T;
      },
      rs_lds);
  if (res != list) {
    const int total = start[T];
    for (int e = tid; e < total; e += kKnnBwdThreads) list[e] = res[e];
  }
}

template <int CG>
__global__ __launch_bounds__(256) void knn_bwd_gather_kernel(
    const float* __restrict__ x1, const float* __restrict__ x2, const float* __restrict__ gd0,
    const int* __restrict__ idx0, const float* __restrict__ gd1, const int* __restrict__ idx1,
    int c, int n, int m, int k, KnnBwdWs ws, float* __restrict__ g1, float* __restrict__ g2) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n + m) return;
  const int side = t < n ? 0 : 1;  // cloud A of this point: 0 = xyz1, 1 = xyz2
  const int i = side ? t - n : t;
  const int Na = side ? m : n, Nb = side ? n : m;
  const float* xa = (side ? x2 : x1) + (size_t)b * c * Na;
  const float* xb = (side ? x1 : x2) + (size_t)b * c * Nb;
  const float* gdo = (side ? gd1 : gd0) + (size_t)b * k * Na;  // own direction
  const int* ido = (side ? idx1 : idx0) + (size_t)b * k * Na;
  const float* gdt = (side ? gd0 : gd1) + (size_t)b * k * Nb;  // cloud B's direction
  const int* lst = ws.list[1 - side] + (size_t)b * k * Nb;
  const int* st = ws.start[1 - side] + (size_t)b * (Na + 1);
  float* out = (side ? g2 : g1) + (size_t)b * c * Na;
  const int s0 = st[i], s1 = st[i + 1];
  for (int c0 = 0; c0 < c; c0 += CG) {
    float acc[CG], xi[CG];
#pragma unroll
    for (int p = 0; p < CG; p++) {
      acc[p] = 0.0f;
      xi[p] = c0 + p < c ? xa[(size_t)(c0 + p) * Na + i] : 0.0f;
    }
    for (int q = 0; q < k; q++) {
      const float g = gdo[(size_t)q * Na + i] * 2.0f;
      const int j = ido[(size_t)q * Na + i];
      if (g >= 20000.0f || j < 0 || j >= Nb) continue;
#pragma unroll
      for (int p = 0; p < CG; p++)
        if (c0 + p < c) acc[p] += g * (xi[p] - xb[(size_t)(c0 + p) * Nb + j]);
    }
    // the pairs naming this point, ascending: four at a time with their
    // loads issued ahead of the in-order sums (a hub point named by
    // thousands of pairs waits a quarter of the load round trips)
    int e = s0;
    for (; e + 4 <= s1; e += 4) {
      int pp[4];
      float g[4], xv[4][CG];
#pragma unroll
      for (int u = 0; u < 4; u++) pp[u] = lst[e + u];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i2 = pp[u] % Nb;
        g[u] = gdt[pp[u]] * 2.0f;
#pragma unroll
        for (int p = 0; p < CG; p++) xv[u][p] = c0 + p < c ? xb[(size_t)(c0 + p) * Nb + i2] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
#pragma unroll
        for (int p = 0; p < CG; p++)
          if (c0 + p < c) acc[p] += -(g[u] * (xv[u][p] - xi[p]));
    }
    for (; e < s1; e++) {
      const int pp = lst[e];
      const int i2 = pp % Nb;
      const float g = gdt[pp] * 2.0f;
#pragma unroll
      for (int p = 0; p < CG; p++)
        if (c0 + p < c) acc[p] += -(g * (xb[(size_t)(c0 + p) * Nb + i2] - xi[p]));
    }
#pragma unroll
    for (int p = 0; p < CG; p++)
      if (c0 + p < c) out[(size_t)(c0 + p) * Na + i] = acc[p];
  }
}

// ppf.cu:28-90
__global__ __launch_bounds__(256) void global_ppf_kernel(const float* __restrict__ coords,
                                                         const float* __restrict__ center,
                                                         const float* __restrict__ normals,
                                                         const float* __restrict__ cnormals, int n,
                                                         float* __restrict__ feat) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t o3 = (size_t)b * 3 * n, o4 = (size_t)b * 4 * n;
  float out[4];
  pcr_global_ppf(coords[o3 + i], coords[o3 + i + n], coords[o3 + i + 2 * n], center[o3 + i],
                 center[o3 + i + n], center[o3 + i + 2 * n], normals[o3 + i],
                 normals[o3 + i + n], normals[o3 + i + 2 * n], cnormals[o3 + i],
                 cnormals[o3 + i + n], cnormals[o3 + i + 2 * n], out);
#pragma unroll
  for (int ch = 0; ch < 4; ch++) feat[o4 + i + (size_t)ch * n] = out[ch];
}

// pvcnn_classify.py:258-269 with explicit neighbour indices; out [b,4,u,m]
// buffer resource over [p, p + bytes): raw buffer loads / stores take a
// 32-bit byte offset (no 64-bit address arithmetic per access)
__device__ inline __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ inline float bld(__amdgpu_buffer_rsrc_t r, unsigned i) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4u), 0, 0));
}

__global__ __launch_bounds__(256) void local_ppf_kernel(
    const float* __restrict__ pts, const float* __restrict__ nrm, const float* __restrict__ ctr,
    const float* __restrict__ cnrm, const int* __restrict__ idx, int n, int m, int u, int kmajor,
    int relative, float* __restrict__ out) {
  const unsigned j = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned q = blockIdx.y;
  const unsigned b = blockIdx.z;
  if (j >= (unsigned)m) return;
  const unsigned un = (unsigned)n, um = (unsigned)m, uu = (unsigned)u;
  const auto P = buf_rsrc(pts + (size_t)b * 3 * un, 12u * un);
  const auto Nn = buf_rsrc(nrm + (size_t)b * 3 * un, 12u * un);
  const auto C = buf_rsrc(ctr + (size_t)b * 3 * um, 12u * um);
  const auto Cn = buf_rsrc(cnrm + (size_t)b * 3 * um, 12u * um);
  const int* I = idx + (size_t)b * um * uu;
  const int si = kmajor ? I[q * um + j] : I[j * uu + q];
  const unsigned s = (si < 0 || si >= n) ? 0u : (unsigned)si;
  float o[4];
  pcr_local_ppf(bld(C, j), bld(C, j + um), bld(C, j + 2 * um), bld(Cn, j), bld(Cn, j + um),
                bld(Cn, j + 2 * um), bld(P, s), bld(P, s + un), bld(P, s + 2 * un), bld(Nn, s),
                bld(Nn, s + un), bld(Nn, s + 2 * un), relative, o);
  float* O = out + (size_t)b * 4 * uu * um;
#pragma unroll
  for (unsigned ch = 0; ch < 4; ch++) O[(ch * uu + q) * um + j] = o[ch];
}

// The same local PPF when the centres are the points themselves and the
// indices are k-major [B, k, N] (the extractor's self-KNN neighbours): one
// workgroup per (cloud, 256 points, SL slots).  The cloud's coordinates and
// normals are staged in LDS in the same round trip as the workgroup's index
// rows, so every neighbour gather is an LDS read: no dependent global loads,
// which under the grid kernel's write stream take microseconds each.
constexpr int kPpfSelfMaxN = 2048;
template <int SL, int NT = 256>
__global__ __launch_bounds__(NT) void local_ppf_self_kernel(const float* __restrict__ xyz,
                                                             const float* __restrict__ nrm,
                                                             const int* __restrict__ idx, int n,
                                                             int k, int relative,
                                                             float* __restrict__ out,
                                                             const int* __restrict__ sidx,
                                                             const int* __restrict__ inv,
                                                             int npad, int* __restrict__ idx_out) {
  extern __shared__ __align__(16) float cl_s[];  // [6][n]: x y z nx ny nz
  (void)PCR_PRIO(2);
  const int tid = threadIdx.x;
  const int j = blockIdx.x * NT + tid;
  const int q0 = blockIdx.y * SL;
  const int b = blockIdx.z;
  const float* P = xyz + (size_t)b * 3 * n;
  const float* Nn = nrm + (size_t)b * 3 * n;
  int id[SL];
  if (sidx) {
    // neighbour ids in the selection's sorted query order: this point's row
    // position from the sort's inverse permutation; the ids are written out
    // in original order here, whole rows (the KNN output knn_idx)
    const int p = j < n ? inv[(size_t)b * n + j] : 0;
#pragma unroll
    for (int s = 0; s < SL; s++)
      id[s] = (j < n && q0 + s < k) ? sidx[((size_t)b * kKnnSortedK + q0 + s) * npad + p] : 0;
#pragma unroll
    for (int s = 0; s < SL; s++)
      if (j < n && q0 + s < k) idx_out[((size_t)b * k + q0 + s) * n + j] = id[s];
  } else {
#pragma unroll
    for (int s = 0; s < SL; s++)
      id[s] = (j < n && q0 + s < k) ? idx[((size_t)b * k + q0 + s) * n + j] : 0;
  }
  constexpr int E = kPpfSelfMaxN / NT;
  float st[E][6];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int i = e * NT + tid;
    if (i < n) {
#pragma unroll
      for (int a = 0; a < 3; a++) {
        st[e][a] = P[(size_t)a * n + i];
        st[e][3 + a] = Nn[(size_t)a * n + i];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int i = e * NT + tid;
    if (i < n)
#pragma unroll
      for (int a = 0; a < 6; a++) cl_s[(size_t)a * n + i] = st[e][a];
  }
  __syncthreads();
  if (j >= n) return;
  const float cx = cl_s[j], cy = cl_s[n + j], cz = cl_s[2 * n + j];
  const float cnx = cl_s[3 * n + j], cny = cl_s[4 * n + j], cnz = cl_s[5 * n + j];
  float* O = out + (size_t)b * 4 * k * n;
#pragma unroll
  for (int s = 0; s < SL; s++) {
    const int q = q0 + s;
    if (q < k) {
      const unsigned si = (id[s] < 0 || id[s] >= n) ? 0u : (unsigned)id[s];
      float o[4];
      pcr_local_ppf(cx, cy, cz, cnx, cny, cnz, cl_s[si], cl_s[n + si], cl_s[2 * n + si],
                    cl_s[3 * n + si], cl_s[4 * n + si], cl_s[5 * n + si], relative, o);
      // nontemporal: the PPF rows are streamed out (c3 KNN + PPF 0.91 -> 0.85 ms)
#pragma unroll
      for (int ch = 0; ch < 4; ch++)
        __builtin_nontemporal_store(o[ch], &O[((size_t)ch * k + q) * n + j]);
    }
  }
}


// The same local PPF from the selection's sorted-order id rows
// (pcr_knn_select_ppf), one workgroup per (cloud, SL slots) covering every
// point of the cloud: the cloud's coordinates + normals and the SL id rows
// (sorted query order, KnnSet::sidx) are staged in LDS by coalesced loads,
// each exactly once per workgroup, and every neighbour / id lookup is an LDS
// read.  The per-256-point workgroups of local_ppf_self_kernel gathered the
// id rows through the sort's inverse permutation from global memory, each
// 4-byte gather on its own line, and the four workgroups of a (cloud, slot
// group) sat on different XCDs, so every XCD's L2 fetched the rows again:
// 44.6 MB of HBM traffic per c2 launch against 21.8 MB algorithmic
// (profiles/r03_pmc_traffic.json).  XCD-aware: the dispatcher deals
// workgroups round-robin over the 8 XCDs, so unit (id % 8) * (U / 8) + id / 8
// puts a cloud's slot groups on one XCD (its cloud is fetched into one L2).
// pcr_local_ppf (include/pcr_math.h) with the same bits, in fewer gfx950
// instructions:
//  - the three IEEE divisions by |d| share one refined reciprocal.  The
//    compiler's f32 division is v_div_scale, v_rcp, two FMA refining the
//    reciprocal, five FMA for the quotient, v_div_fmas and v_div_fixup; with
//    |d| and every nonzero numerator in [2^-60, 2^60] the scales are 1, fmas
//    is a plain FMA and fixup passes the quotient through, so the unscaled
//    sequence below yields the same bits (a zero numerator keeps its signed
//    zero, as fixup does).  A wave with any lane outside that range (|d| = 0
//    for the self pair, NaN, extreme scales) takes the plain divisions.
//  - the acos tails are selects, not branches.
__device__ inline float ppf_acos_sel(float x) {
  const float pio2_hi = 1.57079637e+00f, pio2_lo = -4.37113883e-08f;
  const float pi_hi = 3.14159274e+00f, pi_lo = -8.74227766e-08f;
  const float ax = __builtin_fabsf(x);
  const bool mid = ax <= 0.5f;
  const float s = mid ? x : __builtin_sqrtf((1.0f - ax) * 0.5f);
  const float p = pcr_asinf_core(s);
  const float t2 = 2.0f * p;
  const float rm = pio2_hi - (p - pio2_lo);
  const float rn = pi_hi - (t2 - pi_lo);
  const float rt = x > 0.0f ? t2 : rn;
  return mid ? rm : rt;
}
// |v| in [2^-60, 2^60] (NaN / inf excluded) by one unsigned range test on
// the bits; `zero_ok` also accepts +-0.  Bitwise, so no short-circuit branches.
__device__ inline bool ppf_div_safe(float v, bool zero_ok) {
  const unsigned a = __float_as_uint(v) & 0x7FFFFFFFu;
  constexpr unsigned lo = 0x21800000u, hi = 0x5D800000u;  // 2^-60, 2^60
  return ((a - lo) <= (hi - lo)) | (zero_ok & (a == 0u));
}
__device__ inline float ppf_div_shared(float a, float b, float y) {
  float q = a * y;
  float r = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(r, y, q);
  r = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(r, y, q);
  return a == 0.0f ? a : q;
}
// M pairs of one centre in lockstep (every step written for all M before the
// next), so their dependent chains interleave: the scheduler does not
// interleave whole calls by itself.  c[m] / p[m] = {x, y, z, nx, ny, nz} of
// pair m's centre / neighbour.
template <int M>
__device__ inline void ppf_local_dev(const float (&c)[M][6], const float (&p)[M][6], int relative,
                                     float (&out)[M][4]) {
  float dx[M], dy[M], dz[M], dn[M];
  int safe = 1;  // bitwise ANDs of the range tests: no short-circuit branches
#pragma unroll
  for (int m = 0; m < M; m++) {
    const float gx = relative ? p[m][0] - c[m][0] : p[m][0];
    const float gy = relative ? p[m][1] - c[m][1] : p[m][1];
    const float gz = relative ? p[m][2] - c[m][2] : p[m][2];
    dx[m] = c[m][0] - gx;
    dy[m] = c[m][1] - gy;
    dz[m] = c[m][2] - gz;
  }
#pragma unroll
  for (int m = 0; m < M; m++) dn[m] = __builtin_sqrtf(pcr_sumsq3f(dx[m], dy[m], dz[m]));
#pragma unroll
  for (int m = 0; m < M; m++)
    safe &= (int)ppf_div_safe(dn[m], false) & (int)ppf_div_safe(dx[m], true) &
            (int)ppf_div_safe(dy[m], true) & (int)ppf_div_safe(dz[m], true);
  float ux[M], uy[M], uz[M];
  if (__builtin_expect(__all(safe != 0), 1)) {
    float y[M];
#pragma unroll
    for (int m = 0; m < M; m++) y[m] = __builtin_amdgcn_rcpf(dn[m]);
#pragma unroll
    for (int m = 0; m < M; m++) y[m] = __builtin_fmaf(__builtin_fmaf(-dn[m], y[m], 1.0f), y[m], y[m]);
#pragma unroll
    for (int m = 0; m < M; m++) {
      ux[m] = ppf_div_shared(dx[m], dn[m], y[m]);
      uy[m] = ppf_div_shared(dy[m], dn[m], y[m]);
      uz[m] = ppf_div_shared(dz[m], dn[m], y[m]);
    }
  } else {
#pragma unroll
    for (int m = 0; m < M; m++) {
      ux[m] = dx[m] / dn[m];
      uy[m] = dy[m] / dn[m];
      uz[m] = dz[m] / dn[m];
    }
  }
#pragma unroll
  for (int m = 0; m < M; m++) {
    out[m][0] = pcr_clamp1f(pcr_dot3f(p[m][3], p[m][4], p[m][5], ux[m], uy[m], uz[m]));
    out[m][1] = pcr_clamp1f(pcr_dot3f(c[m][3], c[m][4], c[m][5], ux[m], uy[m], uz[m]));
    out[m][2] = pcr_clamp1f(pcr_dot3f(p[m][3], p[m][4], p[m][5], c[m][3], c[m][4], c[m][5]));
    out[m][3] = dn[m];
  }
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int m = 0; m < M; m++) out[m][a] = ppf_acos_sel(out[m][a]);
}

// LDS layout of local_ppf_cloud_kernel: [3][n] coordinates, [3][n] normals,
// [SL][npad] id rows, each region padded to whole LDS-DMA pieces of width V
struct PpfLds {
  int nrm_off, ids_off, bytes;  // byte offsets / total
};
__host__ __device__ inline PpfLds ppf_lds_layout(int n, int sl, int npad, int v) {
  PpfLds l;
  l.nrm_off = lds_dma_pad(12 * n, v);
  l.ids_off = 2 * l.nrm_off;
  l.bytes = l.ids_off + lds_dma_pad(4 * sl * npad, v);
  return l;
}

template <int SL, int V, int NT = 512>
__global__ __launch_bounds__(NT) void local_ppf_cloud_kernel(const float* __restrict__ xyz,
                                                              const float* __restrict__ nrm, int n,
                                                              int k, int relative,
                                                              float* __restrict__ out,
                                                              const int* __restrict__ sidx,
                                                              const int* __restrict__ inv,
                                                              int npad, int* __restrict__ idx_out,
                                                              int pr) {
  extern __shared__ __align__(16) float cl_s[];  // PpfLds: x y z | nx ny nz | id rows
  constexpr int PT = kPpfSelfMaxN / NT;  // points per thread at most
  const int G = (k + SL - 1) / SL;
  const int U = gridDim.x;
  const int id = blockIdx.x;
  const int u = (U % 8 == 0) ? (id % 8) * (U / 8) + id / 8 : id;
  // unit u = (cloud, slot group, point range): a cloud's units are
  // consecutive, so the XCD-aware order keeps them on one XCD
  const int b = u / (G * pr);
  const int rem = u - b * G * pr;
  const int q0 = (rem / pr) * SL;
  const int span = (n + pr - 1) / pr;  // points of this workgroup's range
  const int j0 = (rem % pr) * span, j1 = min(n, j0 + span);
  const int sl = min(SL, k - q0);
  const int tid = threadIdx.x;
  // this thread's points' rows in sorted order, loaded before the staging
  int p[PT];
#pragma unroll
  for (int e = 0; e < PT; e++) {
    const int j = j0 + e * NT + tid;
    p[e] = j < j1 ? inv[(size_t)b * n + j] : 0;
  }
  // the cloud and the id rows straight into LDS (LDS-DMA: every piece in
  // flight at once, one round trip; a loop of loads and LDS stores waited for
  // each of its ~14 trips in turn)
  const PpfLds L = ppf_lds_layout(n, SL, npad, V);
  const float* nl_s = cl_s + L.nrm_off / 4;
  const int* id_s = (const int*)(cl_s + L.ids_off / 4);
  lds_dma_copy<V>(cl_s, xyz + (size_t)b * 3 * n, 12 * n);
  lds_dma_copy<V>((float*)nl_s, nrm + (size_t)b * 3 * n, 12 * n);
  lds_dma_copy<V>((int*)id_s, sidx + ((size_t)b * kKnnSortedK + q0) * npad, 4 * sl * npad);
  wait_vmcnt<0>();
  __syncthreads();
  float* O = out + (size_t)b * 4 * k * n;
  int* I = idx_out + (size_t)b * k * n;
#pragma unroll
  for (int e = 0; e < PT; e++) {
    const int j = j0 + e * NT + tid;
    if (j >= j1) break;
    const float cx = cl_s[j], cy = cl_s[n + j], cz = cl_s[2 * n + j];
    const float cnx = nl_s[j], cny = nl_s[n + j], cnz = nl_s[2 * n + j];
    // the SL slots in lockstep (slots past sl compute on neighbour 0 and are
    // not stored)
    float nb[SL][6];
#pragma unroll
    for (int s = 0; s < SL; s++) {
      const int jd = s < sl ? id_s[s * npad + p[e]] : 0;
      if (s < sl) I[(size_t)(q0 + s) * n + j] = jd;
      const unsigned si = (jd < 0 || jd >= n) ? 0u : (unsigned)jd;
      nb[s][0] = cl_s[si];
      nb[s][1] = cl_s[n + si];
      nb[s][2] = cl_s[2 * n + si];
      nb[s][3] = nl_s[si];
      nb[s][4] = nl_s[n + si];
      nb[s][5] = nl_s[2 * n + si];
    }
    float ce[SL][6], o[SL][4];
#pragma unroll
    for (int s = 0; s < SL; s++) {
      ce[s][0] = cx;
      ce[s][1] = cy;
      ce[s][2] = cz;
      ce[s][3] = cnx;
      ce[s][4] = cny;
      ce[s][5] = cnz;
    }
    ppf_local_dev<SL>(ce, nb, relative, o);
    // nontemporal: the PPF rows are streamed out
#pragma unroll
    for (int s = 0; s < SL; s++)
      if (s < sl)
#pragma unroll
        for (int ch = 0; ch < 4; ch++)
          __builtin_nontemporal_store(o[s][ch], &O[((size_t)ch * k + q0 + s) * n + j]);
  }
}

// The same with four consecutive points per thread and one slot (needs n %
// 4 == 0 and 16-byte aligned rows): every output store is a 16-byte vector
// (five per thread instead of twenty 4-byte stores, the id row included), and
// the four pairs run in lockstep.  Work item f = (slot s, quad qd) of the
// workgroup's SL slots x span / 4 quads, taken in turn by its threads.
typedef float ppf_f4 __attribute__((ext_vector_type(4)));
typedef int ppf_i4 __attribute__((ext_vector_type(4)));
template <int SL, int NT = 512>
__global__ __launch_bounds__(NT) void local_ppf_quad_kernel(const float* __restrict__ xyz,
                                                             const float* __restrict__ nrm, int n,
                                                             int k, int relative,
                                                             float* __restrict__ out,
                                                             const int* __restrict__ sidx,
                                                             const int* __restrict__ inv,
                                                             int npad, int* __restrict__ idx_out,
                                                             int pr) {
  extern __shared__ __align__(16) float cl_s[];  // PpfLds: x y z | nx ny nz | id rows
  const int G = (k + SL - 1) / SL;
  const int U = gridDim.x;
  const int id = blockIdx.x;
  const int u = (U % 8 == 0) ? (id % 8) * (U / 8) + id / 8 : id;
  const int b = u / (G * pr);
  const int rem = u - b * G * pr;
  const int q0 = (rem / pr) * SL;
  const int span = ((n + pr - 1) / pr + 3) & ~3;  // whole quads
  const int j0 = (rem % pr) * span, j1 = min(n, j0 + span);
  const int nq = (j1 - j0) >> 2;
  const int sl = min(SL, k - q0);
  const int tid = threadIdx.x;
  const PpfLds L = ppf_lds_layout(n, SL, npad, 16);
  const float* nl_s = cl_s + L.nrm_off / 4;
  const int* id_s = (const int*)(cl_s + L.ids_off / 4);
  lds_dma_copy<16>(cl_s, xyz + (size_t)b * 3 * n, 12 * n);
  lds_dma_copy<16>((float*)nl_s, nrm + (size_t)b * 3 * n, 12 * n);
  lds_dma_copy<16>((int*)id_s, sidx + ((size_t)b * kKnnSortedK + q0) * npad, 4 * sl * npad);
  wait_vmcnt<0>();
  __syncthreads();
  float* O = out + (size_t)b * 4 * k * n;
  int* I = idx_out + (size_t)b * k * n;
  const int* pinv = inv + (size_t)b * n;
  for (int f = tid; f < sl * nq; f += NT) {
    const int s = f / nq;
    const int j = j0 + 4 * (f - s * nq);
    const int q = q0 + s;
    // the quad's rows in sorted order (inv), its ids, centres and neighbours
    const int4 pv = *(const int4*)(pinv + j);
    const int pp[4] = {pv.x, pv.y, pv.z, pv.w};
    int jd[4];
    float ce[4][6], nb[4][6], o[4][4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
      jd[m] = id_s[s * npad + pp[m]];
      const unsigned si = (jd[m] < 0 || jd[m] >= n) ? 0u : (unsigned)jd[m];
      nb[m][0] = cl_s[si];
      nb[m][1] = cl_s[n + si];
      nb[m][2] = cl_s[2 * n + si];
      nb[m][3] = nl_s[si];
      nb[m][4] = nl_s[n + si];
      nb[m][5] = nl_s[2 * n + si];
    }
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float4 cv = *(const float4*)(cl_s + a * n + j);
      const float4 nv = *(const float4*)(nl_s + a * n + j);
      ce[0][a] = cv.x;
      ce[1][a] = cv.y;
      ce[2][a] = cv.z;
      ce[3][a] = cv.w;
      ce[0][3 + a] = nv.x;
      ce[1][3 + a] = nv.y;
      ce[2][3 + a] = nv.z;
      ce[3][3 + a] = nv.w;
    }
    __builtin_nontemporal_store(ppf_i4{jd[0], jd[1], jd[2], jd[3]}, (ppf_i4*)(I + (size_t)q * n + j));
    ppf_local_dev<4>(ce, nb, relative, o);
#pragma unroll
    for (int ch = 0; ch < 4; ch++)
      __builtin_nontemporal_store(ppf_f4{o[0][ch], o[1][ch], o[2][ch], o[3][ch]},
                                  (ppf_f4*)(O + ((size_t)ch * k + q) * n + j));
  }
}

// ball_query.cu:30-49: points staged through LDS tiles; per-centre early exit
constexpr int kBqTile = 1024;
__global__ __launch_bounds__(256) void ball_query_kernel(const float* __restrict__ centers,
                                                         const float* __restrict__ points, int m,
                                                         int n, float r2, int u,
                                                         int* __restrict__ idx) {
  __shared__ float tile_s[3 * kBqTile];
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < m;
  const float* C = centers + (size_t)b * 3 * m;
  const float* P = points + (size_t)b * 3 * n;
  int* I = idx + (size_t)b * m * u + (size_t)j * u;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  if (active) {
    cx = C[j];
    cy = C[j + m];
    cz = C[j + 2 * m];
  }
  int cnt = 0, first = 0;
  bool done = !active;
  for (int t0 = 0; t0 < n; t0 += kBqTile) {
    if (!__syncthreads_or(!done)) break;
    const int tl = min(kBqTile, n - t0);
    for (int t = threadIdx.x; t < tl; t += blockDim.x) {
      tile_s[t] = P[t0 + t];
      tile_s[kBqTile + t] = P[n + t0 + t];
      tile_s[2 * kBqTile + t] = P[2 * n + t0 + t];
    }
    __syncthreads();
    if (!done) {
      for (int t = 0; t < tl && cnt < u; t++) {
        const float dx = cx - tile_s[t], dy = cy - tile_s[kBqTile + t],
                    dz = cz - tile_s[2 * kBqTile + t];
        const float d2 = pcr_sumsq3f(dx, dy, dz);
        if (d2 < r2 && (double)d2 > 1e-5) {
          if (cnt == 0) first = t0 + t;
          I[cnt] = t0 + t;
          ++cnt;
        }
      }
      if (cnt >= u) done = true;
    }
    __syncthreads();
  }
  if (active)
    for (int v = cnt; v < u; v++) I[v] = first;
}

// The same query, one wave per 64 centres (lane = centre) and NW waves per
// workgroup.  The cloud is staged in LDS once per workgroup and read as
// broadcast float4s (four candidates per read); the squared distances run
// two candidates per packed instruction in the reference's contraction order
// (pcr_sumsq3f: y*y, then +x*x, then +z*z).  Each wave scans a contiguous
// range of 32-point words and keeps, per centre, one hit bit per point: a
// register word stored once per 32 candidates, no per-hit work.  The output
// pass then turns every centre's bit row into its first u hit indices in
// index order (a popcount prefix over the words, one wave per centre row),
// padded with the first hit (0 if none): the reference's slots, whatever the
// count of hits.  (double)d2 > 1e-5 is evaluated as d2 > 1e-5f: float(1e-5)
// lies below 1e-5, so for every float d2 the two agree.
constexpr int kBqWaves = 4;
template <int NW>
__global__ __launch_bounds__(NW * 64) void ball_query_mask_kernel(
    const float* __restrict__ centers, const float* __restrict__ points, int m, int n, int nwords,
    float r2, int u, int* __restrict__ idx) {
  extern __shared__ __align__(16) unsigned char bq_s[];
  const int npad = nwords * 32;
  float* px = (float*)bq_s;
  float* py = px + npad;
  float* pz = py + npad;
  unsigned* msk = (unsigned*)(pz + npad);  // [nwords][64]: bit i of word w = point 32 w + i
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * kWave;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* P = points + (size_t)b * 3 * n;
  for (int i = tid; i < npad; i += NW * kWave) {
    const bool ok = i < n;
    px[i] = ok ? P[i] : __builtin_nanf("");
    py[i] = ok ? P[n + i] : __builtin_nanf("");
    pz[i] = ok ? P[2 * n + i] : __builtin_nanf("");
  }
  const int j = c0 + lane;
  const bool live = j < m;
  const float* C = centers + (size_t)b * 3 * m;
  const float cx = live ? C[j] : 0.0f, cy = live ? C[m + j] : 0.0f, cz = live ? C[2 * m + j] : 0.0f;
  __syncthreads();
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 cx2 = {cx, cx}, cy2 = {cy, cy}, cz2 = {cz, cz};
  const int wpw = (nwords + NW - 1) / NW;
  const int w0 = min(nwords, wv * wpw), w1 = min(nwords, w0 + wpw);
  for (int w = w0; w < w1; w++) {
    unsigned bits = 0u;
#pragma unroll
    for (int t4 = 0; t4 < 32; t4 += 4) {
      const int t = w * 32 + t4;
      const float4 X = *(const float4*)(px + t);
      const float4 Y = *(const float4*)(py + t);
      const float4 Z = *(const float4*)(pz + t);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const f2 dx = cx2 - (h ? f2{X.z, X.w} : f2{X.x, X.y});
        const f2 dy = cy2 - (h ? f2{Y.z, Y.w} : f2{Y.x, Y.y});
        const f2 dz = cz2 - (h ? f2{Z.z, Z.w} : f2{Z.x, Z.y});
        f2 a = dy * dy;
        a = __builtin_elementwise_fma(dx, dx, a);
        const f2 d = __builtin_elementwise_fma(dz, dz, a);
        bits |= (d[0] < r2 && d[0] > 1e-5f ? 1u : 0u) << (t4 + 2 * h);
        bits |= (d[1] < r2 && d[1] > 1e-5f ? 1u : 0u) << (t4 + 2 * h + 1);
      }
    }
    msk[w * kWave + lane] = bits;
  }
  __syncthreads();
  // output: one wave per centre row; lane l takes word 64 q + l of chunk q
  for (int row = wv; row < kWave; row += NW) {
    const int jj = c0 + row;
    if (jj >= m) break;
    int* I = idx + ((size_t)b * m + jj) * u;
    int base = 0, first = -1;
    for (int q0 = 0; q0 < nwords && base < u; q0 += kWave) {
      const int w = q0 + lane;
      unsigned bits = w < nwords ? msk[w * kWave + row] : 0u;
      const int pc = __popc(bits);
      int incl = pc;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const int o = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += o;
      }
      if (first < 0) {
        const unsigned long long any = __ballot(bits != 0u);
        if (any) {
          const int l0 = __builtin_ctzll(any);
          const unsigned b0 = __shfl(bits, l0, kWave);
          first = (q0 + l0) * 32 + __builtin_ctz(b0);
        }
      }
      int s = base + incl - pc;
      while (bits && s < u) {
        I[s++] = w * 32 + __builtin_ctz(bits);
        bits &= bits - 1u;
      }
      base += __shfl(incl, kWave - 1, kWave);
    }
    const int fill = first < 0 ? 0 : first;
    for (int s = min(base, u) + lane; s < u; s += kWave) I[s] = fill;
  }
}

// grouping.cu:29-35: one thread per output element, coalesced stores
__global__ __launch_bounds__(256) void grouping_kernel(const float* __restrict__ feat,
                                                       const int* __restrict__ idx, int c, int n,
                                                       int m, int u, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over m*u
  const int l = blockIdx.y;
  const int b = blockIdx.z;
  const int64_t mu = (int64_t)m * u;
  if (e >= mu) return;
  const int s = idx[(size_t)b * mu + e];
  const float v = (s >= 0 && s < n) ? feat[((size_t)b * c + l) * n + s] : 0.0f;
  out[((size_t)b * c + l) * mu + e] = v;
}

// grouping.cu:69-76
__global__ __launch_bounds__(256) void grouping_grad_kernel(const float* __restrict__ grad_y,
                                                            const int* __restrict__ idx, int c,
                                                            int n, int m, int u,
                                                            float* __restrict__ grad_x) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int l = blockIdx.y;
  const int b = blockIdx.z;
  const int64_t mu = (int64_t)m * u;
  if (e >= mu) return;
  const int s = idx[(size_t)b * mu + e];
  if (s < 0 || s >= n) return;
  atomicAdd(grad_x + ((size_t)b * c + l) * n + s, grad_y[((size_t)b * c + l) * mu + e]);
}

// ---------------------------------------------------------- self tests
__global__ void selftest_f_kernel(int op, const float* x, const float* y, int n, int aux,
                                  float* of, int* oi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (op) {
    case 0: of[i] = pcr_acosf(x[i]); break;
    case 1: of[i] = pcr_atanf(x[i]); break;
    case 2: of[i] = __builtin_sqrtf(x[i]); break;
    case 3: of[i] = x[i] / y[i]; break;
    case 4: oi[i] = pcr_sph_index(x[i], x[i + n], x[i + 2 * n], aux); break;
    default: break;
  }
}
__global__ void selftest_d_kernel(int op, const double* x, const double* y, int n, double* o) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (op) {
    case 0: o[i] = pcr_acos_d(x[i]); break;
    case 1: o[i] = pcr_atan_d(x[i]); break;
    case 2: o[i] = __builtin_sqrt(x[i]); break;
    case 3: o[i] = x[i] / y[i]; break;
    case 4: o[i] = __builtin_fma(x[i], y[i], x[i]); break;
    default: break;
  }
}

template <bool PPF, int CC>
static pcr_status launch_knn_c(const float* xyz1, const float* xyz2, int b, int c, int n, int m,
                               int k, float* dist, int* idx, const float* normals, int relative,
                               float* ppf, hipStream_t st) {
  dim3 grid(ceil_div(n, kKnnThreads), b);
  if (k <= 16)
    hipLaunchKernelGGL((knn_kernel<16, PPF, CC>), grid, dim3(kKnnThreads), 0, st, xyz1, xyz2, c,
                       n, m, k, dist, idx, normals, relative, ppf);
  else if (k <= 32)
    hipLaunchKernelGGL((knn_kernel<32, PPF, CC>), grid, dim3(kKnnThreads), 0, st, xyz1, xyz2, c,
                       n, m, k, dist, idx, normals, relative, ppf);
  else if (k <= 64)
    hipLaunchKernelGGL((knn_kernel<64, PPF, CC>), grid, dim3(kKnnThreads), 0, st, xyz1, xyz2, c,
                       n, m, k, dist, idx, normals, relative, ppf);
  else if (k <= 128)
    hipLaunchKernelGGL((knn_kernel<128, PPF, CC>), grid, dim3(kKnnThreads), 0, st, xyz1, xyz2, c,
                       n, m, k, dist, idx, normals, relative, ppf);
  else
    return PCR_ERR_UNSUPPORTED;
  return PCR_OK;
}

template <bool PPF>
static pcr_status launch_knn(const float* xyz1, const float* xyz2, int b, int c, int n, int m,
                             int k, float* dist, int* idx, const float* normals, int relative,
                             float* ppf, hipStream_t st) {
  if (c == 3)
    return launch_knn_c<PPF, 3>(xyz1, xyz2, b, c, n, m, k, dist, idx, normals, relative, ppf, st);
  if (PPF) return PCR_ERR_UNSUPPORTED;
  return launch_knn_c<false, kMaxC>(xyz1, xyz2, b, c, n, m, k, dist, idx, normals, relative, ppf,
                                    st);
}

}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_knn_forward(const float* xyz1, const float* xyz2, int b, int c, int n,
                                      int m, int k, float* dist1, float* dist2, int* idx1,
                                      int* idx2, void* workspace, size_t workspace_bytes,
                                      void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 1 && n >= 0 && m >= 0 && k >= 1, "knn_forward: invalid sizes");
  PCR_REQUIRE(dist1 && dist2 && idx1 && idx2, "knn_forward: all four outputs required");
  if (b == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  if (c == 3 && n > 0 && m > 0 &&
      knn_spatial(xyz1, xyz2, b, n, m, k, dist1, idx1, dist2, idx2, nullptr, nullptr, 0, nullptr,
                  workspace, workspace_bytes, xyz1 == xyz2 && n == m, st) == PCR_OK)
    return launch_status("knn_forward");
  if (c <= kMaxC && k <= 128) {
    if (n > 0) launch_knn<false>(xyz1, xyz2, b, c, n, m, k, dist1, idx1, nullptr, 0, nullptr, st);
    if (m > 0) launch_knn<false>(xyz2, xyz1, b, c, m, n, k, dist2, idx2, nullptr, 0, nullptr, st);
  } else {
    if (n > 0)
      hipLaunchKernelGGL(knn_generic_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0, st, xyz1,
                         xyz2, c, n, m, k, dist1, idx1);
    if (m > 0)
      hipLaunchKernelGGL(knn_generic_kernel, dim3(ceil_div(m, 256), b), dim3(256), 0, st, xyz2,
                         xyz1, c, m, n, k, dist2, idx2);
  }
  return launch_status("knn_forward");
}

extern "C" pcr_status pcr_knn_backward(const float* xyz1, const float* xyz2,
                                       const float* graddist1, const float* graddist2,
                                       const int* idx1, const int* idx2, int b, int c, int n,
                                       int m, int k, float* gradxyz1, float* gradxyz2,
                                       void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 1 && n >= 0 && m >= 0 && k >= 1, "knn_backward: invalid sizes");
  if (b == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(gradxyz1, 0, sizeof(float) * (size_t)b * c * n, st) != hipSuccess ||
      hipMemsetAsync(gradxyz2, 0, sizeof(float) * (size_t)b * c * m, st) != hipSuccess)
    return launch_status("knn_backward memset");
  if (n > 0)
    hipLaunchKernelGGL(knn_grad_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0, st, xyz1, xyz2,
                       c, n, m, k, graddist1, idx1, gradxyz1, gradxyz2);
  if (m > 0)
    hipLaunchKernelGGL(knn_grad_kernel, dim3(ceil_div(m, 256), b), dim3(256), 0, st, xyz2, xyz1,
                       c, m, n, k, graddist2, idx2, gradxyz2, gradxyz1);
  return launch_status("knn_backward");
}

// clouds past the LDS counters (or empty ones) take the atomic kernel, which
// needs no workspace
static bool knn_bwd_sorted_applies(int n, int m, int k) {
  return !(n > kKnnBwdMaxT || m > kKnnBwdMaxT || n == 0 || m == 0 ||
           (size_t)k * (n > m ? n : m) >= (1u << 31));
}

extern "C" size_t pcr_knn_backward_workspace_size(int b, int n, int m, int k) {
  if (b <= 0 || n < 0 || m < 0 || k <= 0 || !knn_bwd_sorted_applies(n, m, k)) return 256;
  return knn_bwd_ws_layout(b, n, m, k, nullptr, nullptr);
}

extern "C" pcr_status pcr_knn_backward_ws(const float* xyz1, const float* xyz2,
                                          const float* graddist1, const float* graddist2,
                                          const int* idx1, const int* idx2, int b, int c, int n,
                                          int m, int k, float* gradxyz1, float* gradxyz2,
                                          void* workspace, size_t workspace_bytes,
                                          void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 1 && n >= 0 && m >= 0 && k >= 1,
              "knn_backward_ws: invalid sizes");
  if (b == 0) return PCR_OK;
  // clouds past the LDS counters: the atomic kernel (same contract)
  if (!knn_bwd_sorted_applies(n, m, k))
    return pcr_knn_backward(xyz1, xyz2, graddist1, graddist2, idx1, idx2, b, c, n, m, k,
                            gradxyz1, gradxyz2, stream);
  KnnBwdWs ws;
  const size_t need = knn_bwd_ws_layout(b, n, m, k, &ws, (char*)workspace);
  PCR_REQUIRE(workspace != nullptr && workspace_bytes >= need,
              "knn_backward_ws: workspace too small (%zu < %zu)", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const size_t lds = (size_t)(n > m ? n : m) * 4;
  allow_big_lds(knn_bwd_sort_kernel, lds);
  hipLaunchKernelGGL(knn_bwd_sort_kernel, dim3(b, 2), dim3(kKnnBwdThreads), lds, st, graddist1,
                     idx1, graddist2, idx2, n, m, k, ws);
  const dim3 grid(ceil_div(n + m, 256), b);
  if (c <= 3)
    hipLaunchKernelGGL((knn_bwd_gather_kernel<3>), grid, dim3(256), 0, st, xyz1, xyz2, graddist1,
                       idx1, graddist2, idx2, c, n, m, k, ws, gradxyz1, gradxyz2);
  else
    hipLaunchKernelGGL((knn_bwd_gather_kernel<4>), grid, dim3(256), 0, st, xyz1, xyz2, graddist1,
                       idx1, graddist2, idx2, c, n, m, k, ws, gradxyz1, gradxyz2);
  return launch_status("knn_backward_ws");
}

extern "C" pcr_status pcr_knn_local_ppf(const float* xyz, const float* normals, int b, int n,
                                        int k, int relative, int* idx, float* dist, float* ppf,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && k >= 1 && k <= 128, "knn_local_ppf: invalid sizes (k<=128)");
  PCR_REQUIRE(ppf != nullptr && idx != nullptr, "knn_local_ppf: idx and ppf outputs required");
  if (b == 0) return PCR_OK;
  if (knn_spatial(xyz, xyz, b, n, n, k, dist, idx, nullptr, nullptr, normals, normals, relative,
                  ppf, workspace, workspace_bytes, true, as_stream(stream)) == PCR_OK)
    return launch_status("knn_local_ppf");
  launch_knn<true>(xyz, xyz, b, 3, n, n, k, dist, idx, normals, relative, ppf, as_stream(stream));
  return launch_status("knn_local_ppf");
}

extern "C" pcr_status pcr_knn_prepare(const float* xyz, int b, int n, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1, "knn_prepare: invalid sizes");
  if (b == 0) return PCR_OK;
  const pcr_status rc = knn_spatial(xyz, xyz, b, n, n, 1, nullptr, nullptr, nullptr, nullptr,
                                    nullptr, nullptr, 0, nullptr, workspace, workspace_bytes, true,
                                    as_stream(stream), 1);
  if (rc == PCR_ERR_UNSUPPORTED) {
    set_error("knn_prepare: no sorted path for n=%d (use pcr_knn_local_ppf)", n);
    return rc;
  }
  return launch_status("knn_prepare");
}

extern "C" pcr_status pcr_knn_local_ppf_prepared(const float* xyz, const float* normals, int b,
                                                 int n, int k, int relative, int* idx, float* dist,
                                                 float* ppf, const void* workspace,
                                                 size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && k >= 1 && k <= 128,
              "knn_local_ppf_prepared: invalid sizes (k<=128)");
  PCR_REQUIRE(idx != nullptr, "knn_local_ppf_prepared: idx required");
  if (b == 0) return PCR_OK;
  const pcr_status rc = knn_spatial(xyz, xyz, b, n, n, k, dist, idx, nullptr, nullptr, normals,
                                    normals, relative, ppf, const_cast<void*>(workspace),
                                    workspace_bytes, true, as_stream(stream), 2);
  if (rc == PCR_ERR_UNSUPPORTED) {
    set_error("knn_local_ppf_prepared: no sorted path for n=%d, k=%d", n, k);
    return rc;
  }
  return launch_status("knn_local_ppf_prepared");
}

// Selection + local PPF of a prepared (sorted) workspace with the neighbour
// ids passed in sorted query order (knn_spatial stage 4): the selection
// writes whole rows of the workspace, the PPF kernel reads them back through
// the sort's inverse permutation and writes knn_idx [b,k,n] in original
// order together with the PPF [b,4,k,n].  Shapes outside that path (k > 32,
// clouds of more than 2048 points, no sorted views) take the two calls it
// replaces, with the same outputs.
// The two launches of pcr_knn_select_ppf as entry points of their own (the
// c3 bench times the selection in step between them).  select_sorted returns
// PCR_ERR_UNSUPPORTED, launching nothing, when the sorted-rows path does not
// apply (k > 32, clouds of more than 2048 points, no sorted views).
extern "C" pcr_status pcr_knn_select_sorted(const float* xyz, int b, int n, int k,
                                            const void* workspace, size_t workspace_bytes,
                                            void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && k >= 1 && k <= 128, "knn_select_sorted: invalid sizes");
  if (b == 0) return PCR_OK;
  const int* sidx = nullptr;
  const int* inv = nullptr;
  int npad = 0;
  if (workspace == nullptr || n > kPpfSelfMaxN ||
      !knn_sorted_views(const_cast<void*>(workspace), b, n, &sidx, &inv, &npad))
    return PCR_ERR_UNSUPPORTED;
  return knn_spatial(xyz, xyz, b, n, n, k, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                     0, nullptr, const_cast<void*>(workspace), workspace_bytes, true,
                     as_stream(stream), 2 | 4);
}

extern "C" pcr_status pcr_knn_ppf_sorted(const float* xyz, const float* normals, int b, int n,
                                         int k, int relative, int* idx, float* ppf,
                                         const void* workspace, size_t workspace_bytes,
                                         void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && k >= 1 && k <= kKnnSortedK && n <= kPpfSelfMaxN,
              "knn_ppf_sorted: invalid sizes (k <= 32, n <= 2048)");
  PCR_REQUIRE(idx != nullptr && ppf != nullptr, "knn_ppf_sorted: idx and ppf required");
  if (b == 0) return PCR_OK;
  const int* sidx = nullptr;
  const int* inv = nullptr;
  int npad = 0;
  PCR_REQUIRE(workspace != nullptr && workspace_bytes >= pcr_knn_workspace_size(b, n, n) &&
                  knn_sorted_views(const_cast<void*>(workspace), b, n, &sidx, &inv, &npad),
              "knn_ppf_sorted: workspace without sorted neighbour rows");
  // clouds of <= 1024 points: one workgroup per (cloud, 2 slots, 512
  // points), 256 threads of four points each (round 6: 2 slots x 256 threads
  // rather than 4 x 512, twice the workgroups -- c2 +0.5%, pairs +2%, c3
  // within noise, profiles/r06_ab_ppf_shape.log; 4 slots over 256-point
  // ranges was slower).  At 2048 points splitting a workgroup's points
  // re-stages the 48 KB cloud per range (c3: 100 -> 160 us), so those keep
  // one workgroup per (cloud, 2 slots).
  constexpr int SL = 2;
  constexpr int NT = 256;
  const int pr = n <= 1024 ? ceil_div(n, 512) : 1;
  // 16-byte LDS-DMA pieces and output vectors when every row is 16-byte
  // aligned: four points per thread (local_ppf_quad_kernel)
  const bool v16 = n % 4 == 0 && npad % 4 == 0 &&
                   (((uintptr_t)xyz | (uintptr_t)normals | (uintptr_t)sidx | (uintptr_t)inv |
                     (uintptr_t)idx | (uintptr_t)ppf) & 15) == 0;
  const dim3 grid(b * ceil_div(k, SL) * pr);
  if (v16) {
    const size_t lds = ppf_lds_layout(n, SL, npad, 16).bytes;
    allow_big_lds(local_ppf_quad_kernel<SL, NT>, lds);
    hipLaunchKernelGGL((local_ppf_quad_kernel<SL, NT>), grid, dim3(NT), lds, as_stream(stream),
                       xyz, normals, n, k, relative, ppf, sidx, inv, npad, idx, pr);
  } else {
    const size_t lds = ppf_lds_layout(n, SL, npad, 4).bytes;
    allow_big_lds(local_ppf_cloud_kernel<SL, 4>, lds);
    hipLaunchKernelGGL((local_ppf_cloud_kernel<SL, 4>), grid, dim3(512), lds, as_stream(stream),
                       xyz, normals, n, k, relative, ppf, sidx, inv, npad, idx, pr);
  }
  return launch_status("knn_ppf_sorted");
}

// Selection + local PPF of a prepared (sorted) workspace with the neighbour
// ids passed in sorted query order (knn_spatial stage 4): the selection
// writes whole rows of the workspace, the PPF kernel reads them back through
// the sort's inverse permutation and writes knn_idx [b,k,n] in original
// order together with the PPF [b,4,k,n].  Shapes outside that path (k > 32,
// clouds of more than 2048 points, no sorted views) take the two calls it
// replaces, with the same outputs.
extern "C" pcr_status pcr_knn_select_ppf(const float* xyz, const float* normals, int b, int n,
                                         int k, int relative, int* idx, float* ppf,
                                         const void* workspace, size_t workspace_bytes,
                                         void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && k >= 1 && k <= 128, "knn_select_ppf: invalid sizes (k<=128)");
  PCR_REQUIRE(idx != nullptr && ppf != nullptr, "knn_select_ppf: idx and ppf required");
  if (b == 0) return PCR_OK;
  const pcr_status rs = pcr_knn_select_sorted(xyz, b, n, k, workspace, workspace_bytes, stream);
  if (rs == PCR_OK)
    return pcr_knn_ppf_sorted(xyz, normals, b, n, k, relative, idx, ppf, workspace,
                              workspace_bytes, stream);
  const pcr_status rc = pcr_knn_local_ppf_prepared(xyz, normals, b, n, k, relative, idx, nullptr,
                                                   nullptr, workspace, workspace_bytes, stream);
  if (rc != PCR_OK) return rc;
  return pcr_local_ppf_forward(xyz, normals, xyz, normals, idx, b, n, n, k, 1, relative, ppf,
                               stream);
}

extern "C" pcr_status pcr_spherical_ppf_forward(const float* coords, const float* center,
                                                const float* normals, const float* center_normal,
                                                int b, int n, float* feat, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 0, "spherical_ppf_forward: invalid sizes");
  if (b == 0 || n == 0) return PCR_OK;
  hipLaunchKernelGGL(global_ppf_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0,
                     as_stream(stream), coords, center, normals, center_normal, n, feat);
  return launch_status("spherical_ppf_forward");
}

extern "C" pcr_status pcr_local_ppf_forward(const float* points, const float* normals,
                                            const float* centers, const float* center_normals,
                                            const int* idx, int b, int n, int m, int u,
                                            int idx_kmajor, int relative, float* out,
                                            void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1 && m >= 0 && u >= 0, "local_ppf_forward: invalid sizes");
  PCR_REQUIRE(u <= 65535, "local_ppf_forward: u too large");
  if (b == 0 || m == 0 || u == 0) return PCR_OK;
  PCR_PRIO_INIT();
  if (points == centers && normals == center_normals && n == m && idx_kmajor &&
      n <= kPpfSelfMaxN) {
#define PCR_PPF_SELF(SLV)                                                                     \
  hipLaunchKernelGGL((local_ppf_self_kernel<SLV>), dim3(ceil_div(n, 256), ceil_div(u, SLV), b), \
                     dim3(256), (size_t)6 * n * 4, as_stream(stream), points, normals, idx, n,  \
                     u, relative, out, nullptr, nullptr, 0, nullptr)
    PCR_PPF_SELF(8);
#undef PCR_PPF_SELF
    return launch_status("local_ppf_forward");
  }
  hipLaunchKernelGGL(local_ppf_kernel, dim3(ceil_div(m, 256), u, b), dim3(256), 0,
                     as_stream(stream), points, normals, centers, center_normals, idx, n, m, u,
                     idx_kmajor, relative, out);
  return launch_status("local_ppf_forward");
}

extern "C" pcr_status pcr_ball_query(const float* centers, const float* points, int b, int m,
                                     int n, float radius, int u, int* idx, void* stream) {
  PCR_REQUIRE(b >= 0 && m >= 0 && n >= 0 && u >= 1, "ball_query: invalid sizes");
  if (b == 0 || m == 0) return PCR_OK;
  const float r2 = radius * radius;  // ball_query.cpp:24 (float * float)
  const int nwords = (n + 31) / 32;
  // staged cloud (12 B per point) + hit bits (64 centres x 1 bit per point)
  const size_t smem = (size_t)nwords * 32 * 12 + (size_t)nwords * kWave * 4;
  if (n >= 1 && smem <= 96 * 1024) {
    allow_big_lds(ball_query_mask_kernel<kBqWaves>, smem);
    hipLaunchKernelGGL(ball_query_mask_kernel<kBqWaves>, dim3(ceil_div(m, kWave), b),
                       dim3(kBqWaves * kWave), smem, as_stream(stream), centers, points, m, n,
                       nwords, r2, u, idx);
  } else {
    hipLaunchKernelGGL(ball_query_kernel, dim3(ceil_div(m, 256), b), dim3(256), 0,
                       as_stream(stream), centers, points, m, n, r2, u, idx);
  }
  return launch_status("ball_query");
}

extern "C" pcr_status pcr_grouping_forward(const float* features, const int* indices, int b, int c,
                                           int n, int m, int u, float* out, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && m >= 0 && u >= 0, "grouping_forward: invalid sizes");
  PCR_REQUIRE(c <= 65535, "grouping_forward: c too large");
  const int64_t mu = (int64_t)m * u;
  if (b == 0 || c == 0 || mu == 0) return PCR_OK;
  hipLaunchKernelGGL(grouping_kernel, dim3((unsigned)ceil_div64(mu, 256), c, b), dim3(256), 0,
                     as_stream(stream), features, indices, c, n, m, u, out);
  return launch_status("grouping_forward");
}

extern "C" pcr_status pcr_grouping_backward(const float* grad_y, const int* indices, int b, int c,
                                            int n, int m, int u, float* grad_x, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && m >= 0 && u >= 0, "grouping_backward: invalid sizes");
  PCR_REQUIRE(c <= 65535, "grouping_backward: c too large");
  if (b == 0 || c == 0) return PCR_OK;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(grad_x, 0, sizeof(float) * (size_t)b * c * n, st) != hipSuccess)
    return launch_status("grouping_backward memset");
  const int64_t mu = (int64_t)m * u;
  if (mu == 0) return PCR_OK;
  hipLaunchKernelGGL(grouping_grad_kernel, dim3((unsigned)ceil_div64(mu, 256), c, b), dim3(256),
                     0, st, grad_y, indices, c, n, m, u, grad_x);
  return launch_status("grouping_backward");
}

extern "C" pcr_status pcr_selftest_math(int op, const float* x, const float* y, int n, int aux,
                                        float* out_f, int* out_i, void* stream) {
  PCR_REQUIRE(n >= 0 && op >= 0 && op <= 4, "selftest_math: invalid args");
  if (n == 0) return PCR_OK;
  hipLaunchKernelGGL(selftest_f_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream),
                     op, x, y, n, aux, out_f, out_i);
  return launch_status("selftest_math");
}

extern "C" pcr_status pcr_selftest_math_d(int op, const double* x, const double* y, int n,
                                          double* out, void* stream) {
  PCR_REQUIRE(n >= 0 && op >= 0 && op <= 4, "selftest_math_d: invalid args");
  if (n == 0) return PCR_OK;
  hipLaunchKernelGGL(selftest_d_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream),
                     op, x, y, n, out);
  return launch_status("selftest_math_d");
}
