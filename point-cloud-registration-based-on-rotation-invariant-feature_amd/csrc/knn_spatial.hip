// knn_spatial.hip -- exact k-nearest-neighbour search with spatial pruning,
// for gfx950.  Same results as knn/knn.cu:5-49 of the reference (k
// lexicographically smallest (squared distance, index) pairs with distance
// < 10000, squared distance with the reference's FMA contraction, unfilled
// slots (10000, 0)), but sub-quadratic in practice:
//
//  1. knn_sort_kernel -- one workgroup per (cloud, point set): 30-bit Morton
//     code of every point in the cloud's bounding box, LDS bitonic sort of
//     (code, index), then the sorted SoA coordinates + original indices and
//     the axis-aligned box of every 64-point block.
//  2. knn_block_kernel -- one wave per 64 consecutive (Morton-sorted) queries,
//     top-k per lane in registers as a lexicographically sorted array.
//     Candidate blocks are visited outward from the wave's own block; a block
//     is skipped when, for every lane, the squared distance to its box
//     (computed with the same rounding chain, hence a true lower bound of
//     every candidate distance inside) exceeds the lane's current k-th
//     distance.  Candidates of a processed block are loaded once (coalesced,
//     one per lane) and broadcast with v_readlane.  Because the array is kept
//     in (d, index) order, the visiting order cannot change the result.
#include "common.hpp"

namespace pcr {

constexpr int kKnnMaxSortN = 4096;        // single-workgroup LDS sort up to here
constexpr int kSmallSortThreads = 256;
constexpr int kSmallSortN = kSmallSortThreads * kMaxE;
constexpr int kKnnMaxN = 1 << 22;         // global counting sort beyond
constexpr int kBigCellBits = 15;          // top Morton bits of the global sort (32^3 cells)
constexpr int kBigCells = 1 << kBigCellBits;
constexpr int kBlk = 64;


struct KnnSet {
  float* x;   // [b][npad] sorted coordinates (NaN padding)
  float* y;
  float* z;
  int* j;     // [b][npad] original index (-1 padding)
  float* box; // [b][nblk][8] min xyz, max xyz, -, -
  // clouds of more than kKnnMaxSortN points (global counting sort):
  int* cell;     // [b][kBigCells] counts, then starts
  int* pcell;    // [b][n] cell of each point
  int* pslot;    // [b][n] arrival slot inside the cell
  float* frame;  // [b][8] lo xyz, scale xyz
  int* inv;   // [b][n] sorted position of every point (the sort's inverse)
  // clouds of <= kSortedMaxN points (the LDS-cached selection):
  int* sidx;  // [b][kSortedK][npad] neighbour ids in sorted query order
  // larger clouds: the selection's keys, query-major in sorted query order
  double* skey;  // [b][npad][kSkeyK] (d bits << 32 | index), see make_key
  float* rec;    // [b][n][8] x y z nx ny nz - -: the emit kernel's neighbour gathers
  int n, npad, nblk;
};

static inline size_t al256(size_t v) { return (v + 255) / 256 * 256; }

// the cached selection can emit its neighbour ids in sorted (Morton) query
// order -- whole 256-byte rows -- and the local PPF kernel un-permutes them
// while it writes its own outputs (knn_select_ppf_sorted); writing them in
// original order from the selection is one scattered 4-byte store per
// (query, slot): ~7x the write requests of the 4 MB they carry at c2
constexpr int kSortedMaxN = 2048;
constexpr int kSortedK = kKnnSortedK;
// past kSortedMaxN queries the selection writes its k keys per query as one
// contiguous row in sorted query order (a workgroup's 64 rows are one
// contiguous range) and knn_emit_kernel un-permutes them into the outputs:
// writing them from the selection in original order was one scattered
// 4-byte store per (query, slot, output) -- at c5 5 x 134 M stores, which
// slowed the whole launch by ~30%
constexpr int kSkeyK = 64;

static size_t knn_set_layout(int b, int n, KnnSet* s, char* base, size_t off) {
  const int nblk = (n + kBlk - 1) / kBlk;
  const int npad = nblk * kBlk;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off = al256(off + bytes);
    return q;
  };
  float* x = (float*)take((size_t)b * npad * 4);
  float* y = (float*)take((size_t)b * npad * 4);
  float* z = (float*)take((size_t)b * npad * 4);
  int* j = (int*)take((size_t)b * npad * 4);
  float* box = (float*)take((size_t)b * nblk * 8 * 4);
  const bool big = n > kKnnMaxSortN;
  int* cell = big ? (int*)take((size_t)b * kBigCells * 4) : nullptr;
  int* pcell = big ? (int*)take((size_t)b * n * 4) : nullptr;
  int* pslot = big ? (int*)take((size_t)b * n * 4) : nullptr;
  float* frame = big ? (float*)take((size_t)b * 8 * 4) : nullptr;
  const bool sorted_out = n <= kSortedMaxN;
  int* inv = (int*)take((size_t)b * n * 4);
  int* sidx = sorted_out ? (int*)take((size_t)b * kSortedK * npad * 4) : nullptr;
  double* skey = sorted_out ? nullptr : (double*)take((size_t)b * npad * kSkeyK * 8);
  float* rec = (float*)take((size_t)b * n * 8 * 4);
  if (s) {
    s->rec = rec;
    s->inv = inv;
    s->sidx = sidx;
    s->skey = skey;
    s->cell = cell;
    s->pcell = pcell;
    s->pslot = pslot;
    s->frame = frame;
    s->x = x;
    s->y = y;
    s->z = z;
    s->j = j;
    s->box = box;
    s->n = n;
    s->npad = npad;
    s->nblk = nblk;
  }
  return off;
}

__device__ inline unsigned spread10(unsigned v) {
  v &= 0x3FFu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ inline unsigned quant10(float v, float lo, float scale) {
  float t = (v - lo) * scale;
  if (!(t > 0.0f)) return 0u;  // also NaN
  if (t >= 1023.0f) return 1023u;
  return (unsigned)t;
}

template <int NT>
__global__ __launch_bounds__(NT) void knn_sort_kernel(const float* __restrict__ pts, int n,
                                                      int npad_sort, KnnSet s) {
  extern __shared__ __align__(16) unsigned long long keys[];  // [npad_sort]
  __shared__ float red[6][NT / kWave];
  __shared__ float frame[6];
  if (!PCR_PRIO(0)) latency_kernel_priority();
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int E = npad_sort / NT;
  const float* P = pts + (size_t)b * 3 * n;
  float px[kMaxE], py[kMaxE], pz[kMaxE];
  float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int i = e * NT + tid;
    const bool ok = e < E && i < n;
    px[e] = ok ? P[i] : __builtin_nanf("");
    py[e] = ok ? P[n + i] : __builtin_nanf("");
    pz[e] = ok ? P[2 * n + i] : __builtin_nanf("");
    mn[0] = fminf(mn[0], px[e]);  // fminf/fmaxf ignore NaN
    mn[1] = fminf(mn[1], py[e]);
    mn[2] = fminf(mn[2], pz[e]);
    mx[0] = fmaxf(mx[0], px[e]);
    mx[1] = fmaxf(mx[1], py[e]);
    mx[2] = fmaxf(mx[2], pz[e]);
  }
#pragma unroll
  for (int a = 0; a < 3; a++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], off, kWave));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], off, kWave));
    }
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
      red[a][tid >> 6] = mn[a];
      red[3 + a][tid >> 6] = mx[a];
    }
  }
  __syncthreads();
  if (tid < 6) {
    float v = red[tid][0];
    for (int w = 1; w < NT / kWave; w++)
      v = tid < 3 ? fminf(v, red[tid][w]) : fmaxf(v, red[tid][w]);
    frame[tid] = v;
  }
  __syncthreads();
  float lo[3], sc[3];
#pragma unroll
  for (int a = 0; a < 3; a++) {
    lo[a] = frame[a];
    const float ext = frame[3 + a] - frame[a];
    sc[a] = (ext > 0.0f && ext < __builtin_inff()) ? 1023.0f / ext : 0.0f;
  }
  // coarse counting sort on the top 12 Morton bits (16^3 cells).  The order
  // inside a cell is arbitrary: KNN results never depend on the visiting
  // order (keys are compared lexicographically), only its speed does.
  int* hist = (int*)keys;     // [4096]
  int* order = hist + 4096;   // [n]
  // the coordinates in sorted order, written by the scatter from the
  // registers that already hold them: the block pass reads them from LDS
  // instead of gathering P[order[p]] from global memory (a dependent round
  // trip, microseconds under the grid stream's writes)
  float* sxyz = (float*)(order + n);  // [3][n]
  __shared__ int scan_b[NT / kWave + 1];
  for (int c = tid; c < 4096; c += NT) hist[c] = 0;
  __syncthreads();
  int cell[kMaxE], slot[kMaxE];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int i = e * NT + tid;
    cell[e] = -1;
    if (e < E && i < n) {
      const unsigned code = spread10(quant10(px[e], lo[0], sc[0])) |
                            (spread10(quant10(py[e], lo[1], sc[1])) << 1) |
                            (spread10(quant10(pz[e], lo[2], sc[2])) << 2);
      cell[e] = (int)(code >> 18);
      slot[e] = atomicAdd(&hist[cell[e]], 1);
    }
  }
  __syncthreads();
  {
    constexpr int CPT = 4096 / NT;  // bins per thread
    const int c0 = tid * CPT;
    int h[CPT];
    int sum = 0;
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      h[q] = hist[c0 + q];
      sum += h[q];
    }
    const int incl = block_inclusive_scan(sum, scan_b);
    int run = incl - sum;
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      hist[c0 + q] = run;
      run += h[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kMaxE; e++)
    if (cell[e] >= 0) {
      const int pos = hist[cell[e]] + slot[e];
      order[pos] = e * NT + tid;
      sxyz[pos] = px[e];
      sxyz[n + pos] = py[e];
      sxyz[2 * n + pos] = pz[e];
    }
  __syncthreads();
  // sorted SoA + per-block boxes (one wave per block)
  const size_t base = (size_t)b * s.npad;
  const int lane = tid & 63;
  for (int blk = tid >> 6; blk < s.nblk; blk += NT / kWave) {
    const int p = blk * kBlk + lane;
    float x = __builtin_nanf(""), y = x, z = x;
    int j = -1;
    if (p < n) {
      j = order[p];
      x = sxyz[p];
      y = sxyz[n + p];
      z = sxyz[2 * n + p];
      if (s.inv) s.inv[(size_t)b * n + j] = p;
    }
    s.x[base + p] = x;
    s.y[base + p] = y;
    s.z[base + p] = z;
    s.j[base + p] = j;
    float bmn[3] = {x, y, z}, bmx[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; a++) {
      if (p >= n || bmn[a] != bmn[a]) {
        bmn[a] = __builtin_inff();
        bmx[a] = -__builtin_inff();
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        bmn[a] = fminf(bmn[a], __shfl_xor(bmn[a], off, kWave));
        bmx[a] = fmaxf(bmx[a], __shfl_xor(bmx[a], off, kWave));
      }
    }
    if (lane < 8) {
      float v = 0.0f;
      if (lane < 3) v = bmn[lane == 0 ? 0 : (lane == 1 ? 1 : 2)];
      else if (lane < 6) v = bmx[lane == 3 ? 0 : (lane == 4 ? 1 : 2)];
      s.box[((size_t)b * s.nblk + blk) * 8 + lane] = v;
    }
  }
}

// ---- clouds of more than kKnnMaxSortN points: the same coarse Morton
// order through a global counting sort (frame, cell counts, scan, scatter,
// block boxes); order inside a cell arbitrary, as above.
__global__ __launch_bounds__(kSortBlock) void knn_big_frame_kernel(const float* __restrict__ pts,
                                                                   int n, KnnSet s) {
  __shared__ float red[6][kSortBlock / kWave];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* P = pts + (size_t)b * 3 * n;
  float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int i = tid; i < n; i += kSortBlock) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float v = P[i + (size_t)a * n];
      mn[a] = fminf(mn[a], v);
      mx[a] = fmaxf(mx[a], v);
    }
  }
  int* cnt = s.cell + (size_t)b * kBigCells;
  for (int c = tid; c < kBigCells; c += kSortBlock) cnt[c] = 0;
#pragma unroll
  for (int a = 0; a < 3; a++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], off, kWave));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], off, kWave));
    }
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
      red[a][tid >> 6] = mn[a];
      red[3 + a][tid >> 6] = mx[a];
    }
  }
  __syncthreads();
  if (tid < 3) {
    float lo = red[tid][0], hi = red[3 + tid][0];
    for (int w = 1; w < kSortBlock / kWave; w++) {
      lo = fminf(lo, red[tid][w]);
      hi = fmaxf(hi, red[3 + tid][w]);
    }
    const float ext = hi - lo;
    s.frame[(size_t)b * 8 + tid] = lo;
    s.frame[(size_t)b * 8 + 3 + tid] = (ext > 0.0f && ext < __builtin_inff()) ? 1023.0f / ext : 0.0f;
  }
}

__global__ __launch_bounds__(256) void knn_big_count_kernel(const float* __restrict__ pts, int n,
                                                            KnnSet s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= n) return;
  const float* P = pts + (size_t)b * 3 * n;
  const float* f = s.frame + (size_t)b * 8;
  const unsigned code = spread10(quant10(P[i], f[0], f[3])) |
                        (spread10(quant10(P[i + n], f[1], f[4])) << 1) |
                        (spread10(quant10(P[i + 2 * (size_t)n], f[2], f[5])) << 2);
  const int c = (int)(code >> (30 - kBigCellBits));
  s.pcell[(size_t)b * n + i] = c;
  s.pslot[(size_t)b * n + i] = atomicAdd(&s.cell[(size_t)b * kBigCells + c], 1);
}

__global__ __launch_bounds__(kSortBlock) void knn_big_scan_kernel(KnnSet s) {
  __shared__ int scan_b[kSortBlock / kWave + 1];
  constexpr int CPT = kBigCells / kSortBlock;
  int* cnt = s.cell + (size_t)blockIdx.x * kBigCells;
  const int c0 = threadIdx.x * CPT;
  int sum = 0;
  for (int q = 0; q < CPT; q++) sum += cnt[c0 + q];
  const int incl = block_inclusive_scan(sum, scan_b);
  int run = incl - sum;
  for (int q = 0; q < CPT; q++) {
    const int v = cnt[c0 + q];
    cnt[c0 + q] = run;
    run += v;
  }
}

__global__ __launch_bounds__(256) void knn_big_scatter_kernel(const float* __restrict__ pts, int n,
                                                              KnnSet s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  const size_t base = (size_t)b * s.npad;
  if (i < n) {
    const float* P = pts + (size_t)b * 3 * n;
    const size_t o = base + s.cell[(size_t)b * kBigCells + s.pcell[(size_t)b * n + i]] +
                     s.pslot[(size_t)b * n + i];
    s.x[o] = P[i];
    s.y[o] = P[i + n];
    s.z[o] = P[i + 2 * (size_t)n];
    s.j[o] = i;
    s.inv[(size_t)b * n + i] = (int)(o - base);
  } else if (i < s.npad) {
    s.x[base + i] = s.y[base + i] = s.z[base + i] = __builtin_nanf("");
    s.j[base + i] = -1;
  }
}

// one wave per 64-point block
__global__ __launch_bounds__(256) void knn_big_boxes_kernel(KnnSet s) {
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  if (blk >= s.nblk) return;
  const size_t p = (size_t)b * s.npad + (size_t)blk * kBlk + lane;
  const float v[3] = {s.x[p], s.y[p], s.z[p]};
  float bmn[3], bmx[3];
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const bool real = s.j[p] >= 0 && v[a] == v[a];
    bmn[a] = real ? v[a] : __builtin_inff();
    bmx[a] = real ? v[a] : -__builtin_inff();
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      bmn[a] = fminf(bmn[a], __shfl_xor(bmn[a], off, kWave));
      bmx[a] = fmaxf(bmx[a], __shfl_xor(bmx[a], off, kWave));
    }
  }
  const float bv = lane == 0 ? bmn[0] : lane == 1 ? bmn[1] : lane == 2 ? bmn[2]
                 : lane == 3 ? bmx[0] : lane == 4 ? bmx[1] : lane == 5 ? bmx[2] : 0.0f;
  if (lane < 8) s.box[((size_t)b * s.nblk + blk) * 8 + lane] = bv;
}

// Top-k in registers as packed keys (float bits of the squared distance << 32
// | index).  Squared distances are >= +0 or NaN, so unsigned key order is the
// lexicographic (distance, index) order.  The same 64 bits read as an IEEE
// double have the same order (positive, non-NaN doubles order like their
// bits), so compare-exchanges are one v_min_f64 + one v_max_f64 -- no lane
// masks, no VCC hazards, full ILP -- instead of two 64-bit integer compares
// and four selects.  Keys of NaN distances never enter the array (they fail
// the `< k-th` test).  f64 denormals (distance 0 with small index) are
// preserved by the default float mode.  Valid region = the last k slots; the
// first KMAX-k hold +0.0 and are never displaced.
typedef double kkey;
#define PCR_KEY_PAD 1.7976931348623157e308  // DBL_MAX: above every real key

__device__ inline kkey make_key(float d, int j) {
  // sign cleared: a NaN distance (e.g. a NaN-padded candidate; subtraction
  // flips the NaN's sign) must read as a huge positive key, never negative
  return __longlong_as_double((long long)(((unsigned long long)(__float_as_uint(d) & 0x7FFFFFFFu)
                                           << 32) | (unsigned)j));
}
// a taken key (d below a finite cut: never NaN, and a sum of squares is
// never negative) needs no sign clearing
__device__ inline kkey make_key_finite(float d, int j) {
  return __longlong_as_double(
      (long long)(((unsigned long long)__float_as_uint(d) << 32) | (unsigned)j));
}
__device__ inline float key_dist(kkey k) {
  return __uint_as_float((unsigned)((unsigned long long)__double_as_longlong(k) >> 32));
}
__device__ inline int key_idx(kkey k) {
  return (int)(unsigned)((unsigned long long)__double_as_longlong(k) & 0xFFFFFFFFull);
}

template <int KMAX>
struct TopKKey {
  kkey key[KMAX];
  __device__ void init(int k) {
    const kkey undef = make_key(PCR_KNN_UNDEF, 0);
#pragma unroll
    for (int q = 0; q < KMAX; q++) key[q] = (q < KMAX - k) ? 0.0 : undef;
  }
  __device__ bool qualifies(kkey x) const { return x < key[KMAX - 1]; }
  __device__ float kth() const { return key_dist(key[KMAX - 1]); }
};

__device__ inline void cex_up(kkey& a, kkey& b) {
  const kkey lo = __builtin_fmin(a, b);
  const kkey hi = __builtin_fmax(a, b);
  a = lo;
  b = hi;
}

// Merge a batch of kQ (unsorted) keys into the sorted top-k array: bitonic
// sort of the batch, C[i] = min(A[i], Q[K-1-i]) (the K smallest of A u Q as
// a bitonic sequence), then a bitonic merge.
constexpr int kQ = 8;
template <int KMAX>
__device__ inline void merge_batch(kkey (&key)[KMAX], kkey (&q)[kQ]) {
#pragma unroll
  for (int kk = 2; kk <= kQ; kk <<= 1) {
#pragma unroll
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
#pragma unroll
      for (int i = 0; i < kQ; i++) {
        const int l = i ^ jj;
        if (l > i) {
          if ((i & kk) == 0)
            cex_up(q[i], q[l]);
          else
            cex_up(q[l], q[i]);
        }
      }
    }
  }
#pragma unroll
  for (int i = KMAX - kQ; i < KMAX; i++) key[i] = __builtin_fmin(key[i], q[KMAX - 1 - i]);
#pragma unroll
  for (int jj = KMAX >> 1; jj > 0; jj >>= 1) {
#pragma unroll
    for (int i = 0; i < KMAX; i++) {
      const int l = i ^ jj;
      if (l > i) cex_up(key[i], key[l]);
    }
  }
}

// v, opaque to the optimiser: values derived from it are formed where used.
// knn_wsel_kernel's compaction payloads 64 r + lane are loop invariants the
// compiler otherwise hoists out of the query loop, one VGPR per register r
// (109 -> 91 VGPRs; c2 +1.8%, profiles/r05_wsel_opaque_ab.log)
__device__ inline int pcr_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ inline float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Lower bound of the FMA-chain squared distance from q to any point of box.
__device__ inline float box_lb(float qx, float qy, float qz, const float* bx) {
  const float gx = qx < bx[0] ? bx[0] - qx : (qx > bx[3] ? qx - bx[3] : 0.0f);
  const float gy = qy < bx[1] ? bx[1] - qy : (qy > bx[4] ? qy - bx[4] : 0.0f);
  const float gz = qz < bx[2] ? bx[2] - qz : (qz > bx[5] ? qz - bx[5] : 0.0f);
  float d = gx * gx;
  d = __builtin_fmaf(gy, gy, d);
  d = __builtin_fmaf(gz, gz, d);
  return d;
}

// Waves per query block: the candidate blocks of one 64-query block are
// dealt round-robin to NW waves (more parallelism than one wave per query
// block: B=32 x N=1024 gives only 512 query blocks for 1024 SIMDs), each wave
// keeps its own top-k, and the lists are merged through LDS at the end.
template <int KMAX>
struct KnnNW {
  // waves per query block / waves per workgroup
  static constexpr int value = KMAX <= 32 ? 8 : (KMAX <= 64 ? 2 : 1);
  static constexpr int wg = KMAX <= 32 ? 8 : 4;
};

// r-th block of the visiting order home, home-1, home+1, home-2, ...
__device__ inline int visit_block(int r, int home, int nblk) {
  const int lo = home, hi = nblk - 1 - home;
  const int m2 = lo < hi ? lo : hi;
  if (r == 0) return home;
  if (r <= 2 * m2) {
    const int o = (r + 1) >> 1;
    return (r & 1) ? home - o : home + o;
  }
  const int extra = r - 2 * m2;
  return lo > hi ? home - (m2 + extra) : home + (m2 + extra);
}

template <int KMAX, bool PPF>
__global__ __launch_bounds__(KnnNW<KMAX>::wg * 64) void knn_block_kernel(
    KnnSet qs, KnnSet cs, int k, float* __restrict__ dist, int* __restrict__ idx,
    // fused local PPF: original candidate coords/normals and query normals
    const float* __restrict__ qxyz, const float* __restrict__ qnrm,
    const float* __restrict__ cxyz, const float* __restrict__ cnrm, int relative,
    float* __restrict__ ppf) {
  constexpr int NW = KnnNW<KMAX>::value;
  constexpr int WGW = KnnNW<KMAX>::wg;  // waves per workgroup
  constexpr int QPW = WGW / NW;          // query blocks per workgroup
  // LDS: the per-lane batches (scan phase) and the merge lists (merge / PPF
  // phase) are never live together -> one union
  constexpr int kQBytes = WGW * kQ * kBlk * 8;
  constexpr int kLBytes = NW > 1 ? QPW * (NW / 2) * KMAX * kBlk * 8 : 8;
  __shared__ __align__(16) unsigned char lds_u[kQBytes > kLBytes ? kQBytes : kLBytes];
  kkey* qbuf = (kkey*)lds_u;
  kkey* lst = (kkey*)lds_u;
  __shared__ float thr_s[WGW][kBlk];
  const int b = blockIdx.y;
  const int wv = threadIdx.x >> 6;
  const int w = wv % NW;                       // wave within its query block
  const int qblk = blockIdx.x * QPW + wv / NW;
  const int lane = threadIdx.x & 63;
  const bool live = qblk < qs.nblk;            // wave-uniform
  const size_t qb = (size_t)b * qs.npad + (size_t)(live ? qblk : 0) * kBlk + lane;
  const float qx = qs.x[qb], qy = qs.y[qb], qz = qs.z[qb];
  const int qj = live ? qs.j[qb] : -1;
  TopKKey<KMAX> top;
  top.init(k);
  kkey* myq = qbuf + wv * kQ * kBlk + lane;
  int qn = 0;
  thr_s[wv][lane] = PCR_KNN_UNDEF;
  __syncthreads();
  PCR_STAMP(0);
  int nflush = 0, nproc = 0;
  kkey thr_key = top.key[KMAX - 1];
  auto flush = [&]() {
    kkey qv[kQ];
#pragma unroll
    for (int s = 0; s < kQ; s++) qv[s] = myq[s * kBlk];
#pragma unroll
    for (int s = 0; s < kQ; s++) qv[s] = s < qn ? qv[s] : PCR_KEY_PAD;
    merge_batch<KMAX>(top.key, qv);
    qn = 0;
    nflush++;
    thr_s[wv][lane] = top.kth();  // publish: an upper bound of the final k-th
    thr_key = __builtin_fmin(thr_key, top.key[KMAX - 1]);
  };
  const int gbase = wv - w;  // first wave of this query block
  const float* boxes = cs.box + (size_t)b * cs.nblk * 8;
  const size_t cbase = (size_t)b * cs.npad;
  int home = (int)(((long long)(live ? qblk : 0) * cs.nblk) / qs.nblk);
  if (home >= cs.nblk) home = cs.nblk - 1;
  auto scan_block = [&](int blk) {
    // best bound known to any wave of this query block
    float thr = top.kth();
#pragma unroll
    for (int o = 0; o < NW; o++) thr = fminf(thr, thr_s[gbase + o][lane]);
    // one key bound: below this wave's k-th key and at most the best k-th
    // distance any wave of the query block has published
    thr_key = __builtin_fmin(top.key[KMAX - 1],
                             __longlong_as_double((long long)(((unsigned long long)
                                 __float_as_uint(thr) << 32) | 0xFFFFFFFFull)));
    const float lb = box_lb(qx, qy, qz, boxes + (size_t)blk * 8);
    if (!__any(lb <= thr)) return;  // no lane can gain from this block
    const size_t cp = cbase + (size_t)blk * kBlk + lane;
    const float cx = cs.x[cp], cy = cs.y[cp], cz = cs.z[cp];
    const int cj = cs.j[cp];
    nproc++;
    for (int t = 0; t < kBlk; t += 2) {
      if (__any(qn > kQ - 2)) flush();
      const float sx0 = readlane_f(cx, t), sy0 = readlane_f(cy, t), sz0 = readlane_f(cz, t);
      const float sx1 = readlane_f(cx, t + 1), sy1 = readlane_f(cy, t + 1),
                  sz1 = readlane_f(cz, t + 1);
      const int sj0 = __builtin_amdgcn_readlane(cj, t);
      const int sj1 = __builtin_amdgcn_readlane(cj, t + 1);
      const float a0 = qx - sx0, b0 = qy - sy0, c0 = qz - sz0;
      const float a1 = qx - sx1, b1 = qy - sy1, c1 = qz - sz1;
      float d0 = a0 * a0, d1 = a1 * a1;
      d0 = __builtin_fmaf(b0, b0, d0);
      d1 = __builtin_fmaf(b1, b1, d1);
      d0 = __builtin_fmaf(c0, c0, d0);
      d1 = __builtin_fmaf(c1, c1, d1);
      const kkey k0 = make_key(d0, sj0), k1 = make_key(d1, sj1);
      // keys above this wave's (stale) k-th, or farther than another wave's
      // k-th distance, can never reach the final list.  Branch-free append:
      // slot qn is free (flushed above when fewer than 2 are left).
      myq[qn * kBlk] = k0;
      qn += k0 < thr_key ? 1 : 0;
      myq[qn * kBlk] = k1;
      qn += k1 < thr_key ? 1 : 0;
    }
  };
  // warm-up: wave 0 alone scans the home block and publishes its k-th
  // distance, so the other waves start with a tight bound instead of each
  // filling a list of its own from scratch
  if (live && w == 0) {
    scan_block(home);
    if (__any(qn > 0)) flush();
  }
  if (NW > 1) __syncthreads();
  if (live) {
    for (int rr = (w == 0 ? NW : w); rr < cs.nblk; rr += NW) scan_block(visit_block(rr, home, cs.nblk));
    if (__any(qn > 0)) flush();
  }
  PCR_STAMP(1);
  (void)nflush;
  (void)nproc;
  // merge the NW lists of a query block: tree of bitonic merges through LDS.
  // The partner's k-k front sentinels (key 0) must not enter the result:
  // they read as +inf.
  const int base = KMAX - k;
#pragma unroll
  for (int half = NW / 2; half >= 1; half >>= 1) {
    __syncthreads();
    if (live && w >= half && w < 2 * half) {
      kkey* dst = lst + (size_t)((wv / NW) * (NW / 2) + (w - half)) * KMAX * kBlk;
#pragma unroll
      for (int s = 0; s < KMAX; s++) dst[s * kBlk + lane] = top.key[s];
    }
    __syncthreads();
    if (live && w < half) {
      const kkey* src = lst + (size_t)((wv / NW) * (NW / 2) + w) * KMAX * kBlk;
      // C[i] = min(A[i], B[K-1-i]) then bitonic merge
#pragma unroll
      for (int i = 0; i < KMAX; i++) {
        // partner's reals ascending then padding: B''[t] = B[base + t] (t < k)
        const kkey o = i >= base ? src[(base + KMAX - 1 - i) * kBlk + lane] : PCR_KEY_PAD;
        top.key[i] = __builtin_fmin(top.key[i], o);
      }
#pragma unroll
      for (int jj = KMAX >> 1; jj > 0; jj >>= 1) {
#pragma unroll
        for (int i = 0; i < KMAX; i++) {
          const int l = i ^ jj;
          if (l > i) cex_up(top.key[i], top.key[l]);
        }
      }
    }
  }
  PCR_STAMP(2);
  const int n = qs.n;
  if (live && w == 0 && qj >= 0) {
#pragma unroll
    for (int s = 0; s < KMAX; s++) {
      if (s >= base) {
        const size_t o = ((size_t)b * k + (s - base)) * n + qj;
        if (dist) dist[o] = key_dist(top.key[s]);
        idx[o] = key_idx(top.key[s]);
      }
    }
  }
  if (PPF) {
    // every wave of the query block takes a share of the slots
    kkey* fin = lst + (size_t)(wv / NW) * KMAX * kBlk;
    if (NW > 1) {
      __syncthreads();  // merge reads of lst are complete
      if (live && w == 0) {
#pragma unroll
        for (int s = 0; s < KMAX; s++) fin[s * kBlk + lane] = top.key[s];
      }
      __syncthreads();
    }
    if (!live || qj < 0) return;
    const int m = cs.n;
    const float* cb = cxyz + (size_t)b * 3 * m;
    const float* nb = cnrm + (size_t)b * 3 * m;
    const float* qnr = qnrm + (size_t)b * 3 * n;
    const float* qo = qxyz + (size_t)b * 3 * n;
    const float ox = qo[qj], oy = qo[qj + n], oz = qo[qj + 2 * n];
    const float cnx = qnr[qj], cny = qnr[qj + n], cnz = qnr[qj + 2 * n];
#pragma unroll 1
    for (int slot = w; slot < k; slot += NW) {
      const int jn = NW > 1 ? key_idx(fin[(base + slot) * kBlk + lane])
                            : idx[((size_t)b * k + slot) * n + qj];
      float o[4];
      pcr_local_ppf(ox, oy, oz, cnx, cny, cnz, cb[jn], cb[jn + m], cb[jn + 2 * m], nb[jn],
                    nb[jn + m], nb[jn + 2 * m], relative, o);
#pragma unroll
      for (int ch = 0; ch < 4; ch++) ppf[(((size_t)b * 4 + ch) * k + slot) * n + qj] = o[ch];
    }
  }
}

// ---------------------------------------------------------------------------
// knn_select_kernel (k <= 32): threshold selection instead of per-wave top-k
// lists.  One workgroup of NW waves serves 64 Morton-consecutive queries (one
// per lane); the candidate blocks are dealt round-robin to the waves.  At
// N = 1024 no block can be skipped for a whole 64-query block (the 64 k-NN
// balls cover most of the cloud), so every pass is a brute-force sweep over
// the candidates, two per packed-fp32 instruction.  Clouds of <= kSelCache
// points are staged in LDS once per workgroup and read as broadcast
// ds_read_b128 (in-order LDS returns: no scalar-load round trip in the
// loop); larger ones are read through scalar loads.
//
//  1. bound   D_q = min over candidate blocks holding >= k points of the
//             largest distance from q to the block's box (the same rounding
//             chain, so >= every candidate distance in it): at least k
//             candidates lie within D_q, hence kth(q) <= D_q.
//  2. count   histogram of every candidate distance in quarter-octave bins
//             of d (float bits >> 21) over the kNB bins ending at D_q's bin
//             (bin 0 takes everything below).  One LDS counter per (bin,
//             lane) holds CB-bit fields, one per wave, so the same no-return
//             atomics also give every wave its own counts.
//  3. cut     first bin where the running count reaches k: every candidate
//             with bits >> 21 <= that bin is collected (~1.2-1.9 k for
//             smooth clouds, kCap slots per query).  A wave's slot base is
//             the count of the waves before it, read from the fields.
//  4. collect one sweep writes the (d, index) keys of the collected
//             candidates into the wave's slots.
//  5. rank    the keys are unique; each wave ranks its share of them against
//             all; a key of rank r < k is output slot r.  Every wave then
//             writes k / NW slots and their local PPF (neighbour loads issued
//             for all its slots before any arithmetic).
// A query block where some query has no finite bound below 10000 (fewer than
// k points, NaN / huge coordinates) or more than kCap collected keys
// (duplicates, extreme clustering) takes the exact fallback: wave 0 runs the
// reference's insertion scan with the list in LDS.  Both paths give the
// reference's result: the k lexicographically smallest (d, index) with
// d < 10000, unfilled slots (10000, 0).
constexpr int kNB = 24;
constexpr int kCap = 88;
constexpr int kSelCache = 1024;  // candidates staged in LDS per workgroup
constexpr int kSelMaxK = 32;
constexpr int kCap64 = 112;  // the same selection for 32 < k <= 64 (large clouds): two workgroups per CU
constexpr int kSelMaxK64 = 64;

typedef float pf2 __attribute__((ext_vector_type(2)));

// clamp to [lo, hi] in one instruction (the compiler emits min + max)
__device__ inline int med3_i32(int x, int lo, int hi) {
  int r;
  asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
  return r;
}

// Upper bound of the FMA-chain squared distance from q to any point of box.
__device__ inline float box_ub(float qx, float qy, float qz, const float* bx) {
  const float gx = fmaxf(fabsf(qx - bx[0]), fabsf(qx - bx[3]));
  const float gy = fmaxf(fabsf(qy - bx[1]), fabsf(qy - bx[4]));
  const float gz = fmaxf(fabsf(qz - bx[2]), fabsf(qz - bx[5]));
  float d = gx * gx;
  d = __builtin_fmaf(gy, gy, d);
  d = __builtin_fmaf(gz, gz, d);
  return d;
}

__device__ inline float cand_dist(float qx, float qy, float qz, float sx, float sy, float sz) {
  const float a = qx - sx, bq = qy - sy, c = qz - sz;
  float d = a * a;
  d = __builtin_fmaf(bq, bq, d);
  d = __builtin_fmaf(c, c, d);
  return d;
}

// two candidates at once (v_pk_add / v_pk_mul / v_pk_fma_f32); per element
// the same operations and roundings as cand_dist
__device__ inline pf2 cand_dist2(pf2 qx, pf2 qy, pf2 qz, pf2 sx, pf2 sy, pf2 sz) {
  const pf2 a = qx - sx, bq = qy - sy, c = qz - sz;
  pf2 d = a * a;
  d = __builtin_elementwise_fma(bq, bq, d);
  d = __builtin_elementwise_fma(c, c, d);
  return d;
}

template <int CB>
__device__ inline unsigned field_sum(unsigned v) {
  if (CB == 8) {
    v = (v & 0x00FF00FFu) + ((v >> 8) & 0x00FF00FFu);
    return (v & 0xFFFFu) + (v >> 16);
  }
  return (v & 0xFFFFu) + (v >> 16);
}

template <int NW, int CB, bool CL, bool PPF, int CAP = kCap, int KSEL = kSelMaxK,
          int CACHE = kSelCache>
__global__ __launch_bounds__(NW * 64) void knn_select_kernel(
    KnnSet qs, KnnSet cs, int k, float* __restrict__ dist, int* __restrict__ idx,
    const float* __restrict__ qxyz, const float* __restrict__ qnrm,
    const float* __restrict__ cxyz, const float* __restrict__ cnrm, int relative,
    float* __restrict__ ppf, int sorted_emit) {
  constexpr int FPD = 32 / CB;              // wave fields per counter dword
  constexpr int NG = (NW + FPD - 1) / FPD;  // counter dwords per (bin, lane)
  // the histogram is dead once the cut is chosen: the collected keys reuse it
  constexpr int kHistBytes = NG * (kNB + 1) * kBlk * 4;
  constexpr int kBufBytes = (CAP + 1) * kBlk * 8;  // row CAP: sink of masked writes
  __shared__ __align__(16) unsigned char sel_u[kHistBytes > kBufBytes ? kHistBytes : kBufBytes];
  unsigned* hist_s = (unsigned*)sel_u;
  kkey* buf_s = (kkey*)sel_u;
  __shared__ unsigned dest_s[kBlk];
  __shared__ unsigned cut_s[2 + 2 * NG][kBlk];  // wave 0's cut: bin, count, wave fields (cut, below)
  // cached clouds: the Morton-sorted candidates (the near ones of a query
  // block cluster in a few groups, so few groups are collected) and their
  // point ids as u16, read with the coordinates: the collect pass never
  // waits on an LDS read inside its sweep
  __shared__ __align__(16) float cand_s[CL ? 3 * CACHE : 4];  // x | y | z
  __shared__ __align__(16) unsigned short cand_j[CL ? CACHE : 8];
  __shared__ __align__(16) float cand_w[CL ? 1 : NW][CL ? 4 : 3 * kBlk];  // a block per wave
  (void)PCR_PRIO(1);
  const int b = blockIdx.y;
  const int qblk = blockIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t qb = (size_t)b * qs.npad + (size_t)qblk * kBlk + lane;
  const float qx = qs.x[qb], qy = qs.y[qb], qz = qs.z[qb];
  const int qj = qs.j[qb];
  const bool qlive = qj >= 0;
  const int m = cs.n;
  const int nblk = cs.nblk;
  const float* boxes = cs.box + (size_t)b * nblk * 8;
  const size_t cbase = (size_t)b * cs.npad;
  const pf2 qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};

  for (int i = threadIdx.x; i < NG * (kNB + 1) * kBlk; i += NW * kBlk) hist_s[i] = 0u;
  if (wv == 0) dest_s[lane] = 0x7F800000u;  // +inf
  if (CL) {
    const int np = cs.npad;
    for (int i = threadIdx.x; i < np; i += NW * kBlk) {
      cand_s[i] = cs.x[cbase + i];
      cand_j[i] = (unsigned short)cs.j[cbase + i];
      cand_s[CACHE + i] = cs.y[cbase + i];
      cand_s[2 * CACHE + i] = cs.z[cbase + i];
    }
  }
  // Visit every group of four candidates this wave owns: f(pos, d[4]), pos =
  // sorted position of the group's first candidate.  Cached clouds: wave w
  // owns candidates [64 b + w S, 64 b + w S + S) of every block b (S = 64 /
  // NW), so the candidates near the queries -- the ones the collect pass
  // keeps -- are spread over all waves; no pruning (at <= CACHE points a
  // 64-query block reaches nearly every candidate block).  The next group's
  // LDS reads are issued before f runs, so their wait never covers the LDS
  // atomics / stores f issues.  Larger clouds: whole blocks round-robin over
  // the waves, skipped when no lane's box distance is below `lim`.
  int nvisit = 0;  // candidate blocks this wave processed (diagnostics)
  // Large clouds: the boxes of this wave's blocks (wv + NW (64 j + lane)) sit
  // in registers and reach the whole wave by v_readlane, so the per-block
  // tests never wait on memory; a processed block is loaded one candidate
  // per lane (coalesced) into the wave's LDS slot and read back as
  // broadcast ds_read_b128, as the cached path does.
  constexpr int kBoxJ = 2;
  const bool breg = !CL && nblk <= NW * kBlk * kBoxJ;
  float bl[kBoxJ][6];
#pragma unroll
  for (int j = 0; j < kBoxJ; j++) {
    const int blk = wv + NW * (j * kBlk + lane);
    const bool ok = breg && blk < nblk;
#pragma unroll
    for (int a = 0; a < 6; a++) bl[j][a] = ok ? boxes[(size_t)blk * 8 + a] : 0.0f;
  }
  // the query block's box (scalar loads; the register-box sweep's prefilter)
  float qbx[6];
#pragma unroll
  for (int a = 0; a < 6; a++)
    qbx[a] = breg ? qs.box[((size_t)b * qs.nblk + qblk) * 8 + a] : 0.0f;
  // visits this wave's blocks in order: g(blk, box[6]) (register boxes only)
  auto for_blocks = [&](auto&& g) {
#pragma unroll
    for (int j = 0; j < kBoxJ; j++) {
      for (int l = 0; l < kBlk; l++) {
        const int blk = wv + NW * (j * kBlk + l);
        if (blk >= nblk) return;
        float b6[6];
#pragma unroll
        for (int a = 0; a < 6; a++) b6[a] = readlane_f(bl[j][a], l);
        g(blk, b6);
      }
    }
  };
  int cj_cur = 0;  // original index of candidate `lane` of the block in process
  // register-box path: blocks a count round already visited (excluded from
  // the next round) and whether this visit records its blocks there
  unsigned long long vskip[kBoxJ];
#pragma unroll
  for (int j = 0; j < kBoxJ; j++) vskip[j] = 0ull;
  bool vrecord = false;
  auto visit = [&](float lim, auto want_j, auto&& f) {
    constexpr bool WANT_J = decltype(want_j)::value;
    if (CL) {
      constexpr int S = kBlk / NW;
      constexpr int GPB = S / 4;
      static_assert(S % 4 == 0, "a wave owns whole groups of four");
      static_assert(GPB == 2, "two groups of four per wave and block");
      // one block (two groups) per half iteration; positions advance by a
      // constant, so every read is one base register plus an immediate.
      // Reads past the last block land in the next LDS array (never used).
      // the ids of the wave's 8 candidates (u16) are read with them only
      // when the callback uses them (the collect pass)
      auto rd = [&](int o, float4 (&X)[2], float4 (&Y)[2], float4 (&Z)[2], uint4& J) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          X[h] = *(const float4*)(cand_s + o + 4 * h);
          Y[h] = *(const float4*)(cand_s + CACHE + o + 4 * h);
          Z[h] = *(const float4*)(cand_s + 2 * CACHE + o + 4 * h);
        }
        if (WANT_J) J = *(const uint4*)(cand_j + o);
      };
      auto eval = [&](int o, const float4 (&X)[2], const float4 (&Y)[2], const float4 (&Z)[2],
                      const uint4& J) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const pf2 d0 = cand_dist2(qx2, qy2, qz2, pf2{X[h].x, X[h].y}, pf2{Y[h].x, Y[h].y},
                                    pf2{Z[h].x, Z[h].y});
          const pf2 d1 = cand_dist2(qx2, qy2, qz2, pf2{X[h].z, X[h].w}, pf2{Y[h].z, Y[h].w},
                                    pf2{Z[h].z, Z[h].w});
          const float d[4] = {d0[0], d0[1], d1[0], d1[1]};
          f(o + 4 * h, d, h == 0 ? uint2{J.x, J.y} : uint2{J.z, J.w});
        }
      };
      // ping-pong register sets A / B, no copies: B's reads are issued
      // before A's evaluation (and its LDS atomics / stores) and vice versa
      float4 AX[2], AY[2], AZ[2], BX[2], BY[2], BZ[2];
      uint4 AJ = {0u, 0u, 0u, 0u}, BJ = {0u, 0u, 0u, 0u};
      int o = wv * S;
      rd(o, AX, AY, AZ, AJ);
      for (int blk = 0; blk < nblk; blk += 2, o += 2 * kBlk) {
        rd(o + kBlk, BX, BY, BZ, BJ);
        __builtin_amdgcn_sched_barrier(0);  // reads first, then A's (older) data is waited on
        eval(o, AX, AY, AZ, AJ);
        rd(o + 2 * kBlk, AX, AY, AZ, AJ);
        __builtin_amdgcn_sched_barrier(0);
        if (blk + 1 < nblk) eval(o + kBlk, BX, BY, BZ, BJ);
      }
    } else if (breg) {
      // which of this wave's blocks does any query lane need?  Lane l tests
      // block wv + NW (64 j + l) against the 64 queries (read by v_readlane):
      // one ballot per 64 blocks instead of one box test + ballot per block
      // (up to 64 blocks per wave, i.e. clouds of <= 32k points: one box
      // test + ballot per block is cheaper than the 64-query sweep)
      unsigned long long vm[kBoxJ];
      if (nblk <= NW * kBlk) {
        vm[0] = 0ull;
#pragma unroll
        for (int j = 1; j < kBoxJ; j++) vm[j] = 0ull;
        for (int l = 0; wv + NW * l < nblk; l++) {
          float b6[6];
#pragma unroll
          for (int a = 0; a < 6; a++) b6[a] = readlane_f(bl[0][a], l);
          if (__any(box_lb(qx, qy, qz, b6) < lim)) vm[0] |= 1ull << l;
        }
      } else {
        // lane l tests block wv + NW (64 j + l) against the box of the
        // query block with the largest limit of its queries (the same
        // rounding chain, so it is a lower bound of every query's box
        // distance: a block failing it is needed by no query); only the
        // blocks passing it get the per-query test (one box test + ballot
        // each), instead of a sweep of all 64 queries for every block
        float mlim = lim;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mlim = fmaxf(mlim, __shfl_xor(mlim, off, kWave));
#pragma unroll
        for (int j = 0; j < kBoxJ; j++) {
          const float gx = fmaxf(fmaxf(bl[j][0] - qbx[3], qbx[0] - bl[j][3]), 0.0f);
          const float gy = fmaxf(fmaxf(bl[j][1] - qbx[4], qbx[1] - bl[j][4]), 0.0f);
          const float gz = fmaxf(fmaxf(bl[j][2] - qbx[5], qbx[2] - bl[j][5]), 0.0f);
          float bb = gx * gx;
          bb = __builtin_fmaf(gy, gy, bb);
          bb = __builtin_fmaf(gz, gz, bb);
          unsigned long long cand =
              __ballot(bb < mlim && wv + NW * (j * kBlk + lane) < nblk);
          vm[j] = 0ull;
          while (cand) {
            const int l = __builtin_ctzll(cand);
            cand &= cand - 1ull;
            float b6[6];
#pragma unroll
            for (int a = 0; a < 6; a++) b6[a] = readlane_f(bl[j][a], l);
            if (__any(box_lb(qx, qy, qz, b6) < lim)) vm[j] |= 1ull << l;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < kBoxJ; j++) {
        vm[j] &= ~vskip[j];
        if (vrecord) vskip[j] |= vm[j];
      }
      // the visited blocks in order, the next one's candidates loaded (one
      // per lane) while the current one is evaluated from the wave's LDS slot
      int jc = 0;
      auto next = [&]() {
        while (jc < kBoxJ && vm[jc] == 0ull) jc++;
        if (jc >= kBoxJ) return -1;
        const int l = __builtin_ctzll(vm[jc]);
        vm[jc] &= vm[jc] - 1ull;
        return wv + NW * (jc * kBlk + l);
      };
      float* cw = cand_w[CL ? 0 : wv];
      int cur = next();
      float px = 0.0f, py = 0.0f, pz = 0.0f;
      int pj = 0;
      if (cur >= 0) {
        const size_t cp = cbase + (size_t)cur * kBlk + lane;
        px = cs.x[cp];
        py = cs.y[cp];
        pz = cs.z[cp];
        pj = cs.j[cp];
      }
      while (cur >= 0) {
        nvisit++;
        const int nxt = next();
        // the wave's previous block is fully read (LDS is in order per wave)
        cw[lane] = px;
        cw[kBlk + lane] = py;
        cw[2 * kBlk + lane] = pz;
        cj_cur = pj;
        if (nxt >= 0) {
          const size_t cp = cbase + (size_t)nxt * kBlk + lane;
          px = cs.x[cp];
          py = cs.y[cp];
          pz = cs.z[cp];
          pj = cs.j[cp];
        }
        // ping-pong register sets: the next group's LDS reads are issued
        // before this group's callback (its LDS atomics / stores), so its
        // wait never covers them (LDS operations complete in order)
        auto rd4 = [&](int t, float4& X, float4& Y, float4& Z) __attribute__((always_inline)) {
          X = *(const float4*)(cw + t);
          Y = *(const float4*)(cw + kBlk + t);
          Z = *(const float4*)(cw + 2 * kBlk + t);
        };
        auto ev4 = [&](int t, const float4& X, const float4& Y, const float4& Z)
                       __attribute__((always_inline)) {
          const pf2 d0 = cand_dist2(qx2, qy2, qz2, pf2{X.x, X.y}, pf2{Y.x, Y.y}, pf2{Z.x, Z.y});
          const pf2 d1 = cand_dist2(qx2, qy2, qz2, pf2{X.z, X.w}, pf2{Y.z, Y.w}, pf2{Z.z, Z.w});
          const float d[4] = {d0[0], d0[1], d1[0], d1[1]};
          f(cur * kBlk + t, d, uint2{0u, 0u});
        };
        float4 AX, AY, AZ, BX, BY, BZ;
        rd4(0, AX, AY, AZ);
#pragma unroll 2
        for (int t = 0; t < kBlk; t += 8) {
          rd4(t + 4, BX, BY, BZ);
          __builtin_amdgcn_sched_barrier(0);
          ev4(t, AX, AY, AZ);
          if (t + 8 < kBlk) rd4(t + 8, AX, AY, AZ);
          __builtin_amdgcn_sched_barrier(0);
          ev4(t + 4, BX, BY, BZ);
        }
        cur = nxt;
      }
    } else {
      for (int blk = wv; blk < nblk; blk += NW) {
        if (!__any(box_lb(qx, qy, qz, boxes + (size_t)blk * 8) < lim)) continue;
        nvisit++;
        const float* bx = cs.x + cbase + (size_t)blk * kBlk;
        const float* by = cs.y + cbase + (size_t)blk * kBlk;
        const float* bz = cs.z + cbase + (size_t)blk * kBlk;
#pragma unroll 4
        for (int t = 0; t < kBlk; t += 4) {
          const float4 X = *(const float4*)(bx + t);
          const float4 Y = *(const float4*)(by + t);
          const float4 Z = *(const float4*)(bz + t);
          const pf2 d0 = cand_dist2(qx2, qy2, qz2, pf2{X.x, X.y}, pf2{Y.x, Y.y}, pf2{Z.x, Z.y});
          const pf2 d1 = cand_dist2(qx2, qy2, qz2, pf2{X.z, X.w}, pf2{Y.z, Y.w}, pf2{Z.z, Z.w});
          const float d[4] = {d0[0], d0[1], d1[0], d1[1]};
          f(blk * kBlk + t, d, uint2{0u, 0u});
        }
      }
    }
  };
  // original indices of the four candidates at sorted position pos
  auto cand_idx4 = [&](int pos) {
    if (CL) return int4{0, 0, 0, 0};  // unused: the cached path passes its ids to the callback
    if (breg) {
      const int t = pos & (kBlk - 1);
      return int4{__builtin_amdgcn_readlane(cj_cur, t), __builtin_amdgcn_readlane(cj_cur, t + 1),
                  __builtin_amdgcn_readlane(cj_cur, t + 2),
                  __builtin_amdgcn_readlane(cj_cur, t + 3)};
    }
    const int* bj = cs.j + cbase + pos;
    return int4{bj[0], bj[1], bj[2], bj[3]};
  };
  __syncthreads();
  PCR_STAMP(0);

  // 1. bound
  {
    float dq = __builtin_inff();
    // a self KNN over many blocks takes its bound from the blocks within
    // kBoundWin of the query block in Morton order (any block of >= k points
    // bounds kth, so fewer blocks only loosen the bound; the box nearest a
    // query is almost always there): the boxes are read by scalar loads, not
    // one readlane sweep over all of this wave's blocks
    constexpr int kBoundWin = 64;
    if (!CL && qs.x == cs.x && nblk > 2 * kBoundWin + NW && breg) {
      // the window's boxes of this wave are lanes [l0, l1] of its register
      // boxes (block wv + NW (64 j + l)): v_readlane, no scalar-load chain
      const int lo = max(0, qblk - kBoundWin), hi = min(nblk - 1, qblk + kBoundWin);
#pragma unroll
      for (int j = 0; j < kBoxJ; j++) {
        const int f0 = lo - wv - NW * j * kBlk, f1 = hi - wv - NW * j * kBlk;
        const int l0 = max(0, (f0 + NW - 1 + NW * kBlk) / NW - kBlk), l1 = min(kBlk - 1, f1 >= 0 ? f1 / NW : -1);
        for (int l = l0; l <= l1; l++) {
          const int blk = wv + NW * (j * kBlk + l);
          float b6[6];
#pragma unroll
          for (int a = 0; a < 6; a++) b6[a] = readlane_f(bl[j][a], l);
          if (min(kBlk, m - blk * kBlk) >= k) dq = fminf(dq, box_ub(qx, qy, qz, b6));
        }
      }
    } else if (!CL && qs.x == cs.x && nblk > 2 * kBoundWin + NW) {
      const int lo = max(0, qblk - kBoundWin), hi = min(nblk - 1, qblk + kBoundWin);
      for (int blk = lo + wv; blk <= hi; blk += NW) {
        const int real = min(kBlk, m - blk * kBlk);
        if (real >= k) dq = fminf(dq, box_ub(qx, qy, qz, boxes + (size_t)blk * 8));
      }
    } else if (breg) {
      for_blocks([&](int blk, const float (&b6)[6]) {
        const int real = min(kBlk, m - blk * kBlk);
        if (real >= k) dq = fminf(dq, box_ub(qx, qy, qz, b6));
      });
    } else {
      for (int blk = wv; blk < nblk; blk += NW) {
        const int real = min(kBlk, m - blk * kBlk);
        if (real >= k) dq = fminf(dq, box_ub(qx, qy, qz, boxes + (size_t)blk * 8));
      }
    }
    atomicMin(&dest_s[lane], __float_as_uint(dq));  // NaN never wins: fminf drops it
  }
  __syncthreads();
  const unsigned dbits = dest_s[lane];
  bool fallback = __any(qlive && !(dbits < __float_as_uint(PCR_KNN_UNDEF)));
  const int etop = (int)(dbits >> 21);
  const int ebase = etop - (kNB - 1);
  // smallest distance that is not counted (0 for padding lanes: they never
  // keep a block alive)
  const float ftop = (qlive && !fallback) ? __uint_as_float((unsigned)(etop + 1) << 21) : 0.0f;

  PCR_STAMP(1);
  // 2. count + 3. cut.  Pass 1 counts quarter-octave bins (float bits >> 21)
  // of the kNB below D_q's bin.  A block where some query has more than CAP
  // keys at its cut (a bin of many near-equal distances: an outlier facing
  // the bulk of the cloud) recounts inside each query's cut bin with
  // 1/64-octave bins (bits >> 17) before it gives up to the insertion
  // fallback.  Every wave computes the same cut for its 64 queries.
  // total: keys at or below the cut bin; lo_total (S): keys below it (all of
  // them are among the k nearest); slot / slot_lo: this wave's first slot
  // among all / the below-cut keys of the lane
  int total = 0, slot = 0, bstar = -1, lo_total = 0, slot_lo = 0;
  int shift = 21, base = ebase;
  unsigned ucut = 0u, ulo = 0u;
  auto count_visit = [&](float lim) {
    unsigned* hw = hist_s + (size_t)(wv / FPD) * (kNB + 1) * kBlk + lane;
    const unsigned inc = 1u << ((wv % FPD) * CB);
    // counter of bin e (clamped to [base, base + kNB]; the last = not
    // counted, also NaN) at hwb + e * kBlk
    unsigned* hwb = hw - base * kBlk;
    const int top = base + kNB;
    const int sh = shift;
    visit(lim, std::false_type(), [&](int, const float (&d)[4], uint2) {
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int e = med3_i32((int)(__float_as_uint(d[h]) >> sh), base, top);
        __hip_atomic_fetch_add(hwb + e * kBlk, inc, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    });
  };
  // upper edge of the first bin where the lane's count so far reaches k
  // (every count is a real candidate, so kth(q) lies below it), else `lim`
  auto running_cut = [&](float lim) {
    int cum = 0;
    float t = lim;
    bool found = false;
    for (int bin = 0; bin < kNB; bin++) {
#pragma unroll
      for (int g = 0; g < NG; g++) cum += (int)field_sum<CB>(hist_s[(g * (kNB + 1) + bin) * kBlk + lane]);
      if (!found && cum >= k) {
        found = true;
        t = __uint_as_float((unsigned)(base + bin + 1) << shift);
      }
      if (__all(found)) break;
    }
    return fminf(t, lim);
  };
  auto count_cut = [&](float lim) {
    if (!CL && breg) {
      // large clouds: two rounds.  D_q is several times kth (its bin top
      // reaches past most of the cloud's near blocks), so the blocks near
      // the queries (lower bound below D_q / 8) are counted first; their
      // counts give each query an upper bound of kth (the first bin where
      // the count reaches k), and the second round adds only the blocks
      // below that tighter bound.  Every block a query may need is still
      // counted for it: an unvisited block has every lane's lower bound at
      // or above that lane's limit, and the final cut never exceeds it.
      vrecord = true;
      count_visit(lim * 0.125f);
      vrecord = false;
      __syncthreads();
      count_visit(qlive ? running_cut(lim) : 0.0f);
#pragma unroll
      for (int j = 0; j < kBoxJ; j++) vskip[j] = 0ull;
    } else {
      count_visit(lim);
    }
    __syncthreads();
    PCR_STAMP(2);
    // wave 0 finds the cut of the 64 queries (the other waves would repeat
    // the same sweep) and hands it over through LDS
    unsigned cum[NG], cut[NG], cutb[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) cum[g] = cut[g] = cutb[g] = 0u;
    if (wv == 0) {
      bstar = -1;
      total = 0;
      for (int b0 = 0; b0 < kNB; b0 += 4) {
#pragma unroll
        for (int bin = b0; bin < b0 + 4; bin++) {
          unsigned prev[NG];
          int tb = 0;
#pragma unroll
          for (int g = 0; g < NG; g++) {
            prev[g] = cum[g];
            cum[g] += hist_s[(g * (kNB + 1) + bin) * kBlk + lane];
            tb += (int)field_sum<CB>(cum[g]);
          }
          if (bstar < 0 && tb >= k) {
            bstar = bin;
            total = tb;
#pragma unroll
            for (int g = 0; g < NG; g++) {
              cut[g] = cum[g];
              cutb[g] = prev[g];
            }
          }
        }
        if (__all(bstar >= 0)) break;
      }
      cut_s[0][lane] = (unsigned)bstar;
      cut_s[1][lane] = (unsigned)total;
#pragma unroll
      for (int g = 0; g < NG; g++) {
        cut_s[2 + g][lane] = cut[g];
        cut_s[2 + NG + g][lane] = cutb[g];
      }
    }
    __syncthreads();
    bstar = (int)cut_s[0][lane];
    total = (int)cut_s[1][lane];
#pragma unroll
    for (int g = 0; g < NG; g++) {
      cut[g] = cut_s[2 + g][lane];
      cutb[g] = cut_s[2 + NG + g][lane];
    }
    // slots of the waves before this one, among all and among the below-cut
    // keys; the lane's below-cut total
    const int mg = wv / FPD;
    const unsigned below = (1u << ((wv % FPD) * CB)) - 1u;
    slot = slot_lo = lo_total = 0;
#pragma unroll
    for (int g = 0; g < NG; g++) {
      slot += (int)field_sum<CB>(g < mg ? cut[g] : (g == mg ? (cut[g] & below) : 0u));
      slot_lo += (int)field_sum<CB>(g < mg ? cutb[g] : (g == mg ? (cutb[g] & below) : 0u));
      lo_total += (int)field_sum<CB>(cutb[g]);
    }
  };
  // the collected keys sit in two regions of the key buffer: rows [0, S) the
  // keys below the cut bin (all among the k nearest, S < k), rows [cut0,
  // cut0 + total - S) the cut bin's keys, so each is ranked within its own
  // region (S^2 + C^2 compares instead of (S + C)^2).  A lane whose cut bin
  // holds more than CAP - cut0 keys overflows.
  const int cut0 = (k + 7) & ~7;
  auto overflow = [&]() { return qlive && total - lo_total > CAP - cut0; };
  if (!fallback) {
    count_cut(ftop);
    const bool no_cut = __any(qlive && bstar < 0);
    if (!no_cut && __any(overflow())) {
      // refine: bin 0 = below the cut bin, bins 1..16 = its 16 sub-bins
      const float lim = qlive ? __uint_as_float((unsigned)(base + bstar + 1) << 21) : 0.0f;
      base = qlive ? ((base + bstar) << 4) - 1 : 0;
      shift = 17;
      __syncthreads();  // pass-1 histogram reads done
      for (int i = threadIdx.x; i < NG * (kNB + 1) * kBlk; i += NW * kBlk) hist_s[i] = 0u;
      __syncthreads();
      count_cut(lim);
    }
    fallback = __any(qlive && bstar < 0) || __any(overflow());
    if (qlive && !fallback) {
      ucut = (unsigned)(base + bstar + 1) << shift;
      ulo = bstar > 0 ? (unsigned)(base + bstar) << shift : 0u;
    }
  }
  __syncthreads();  // histogram reads done: buf_s overwrites it
  (void)nvisit;

  if (!fallback) {
    // 4. collect
    const float fcut = __uint_as_float(ucut);
    int slot_cut = cut0 + (slot - slot_lo);
    visit(fcut, std::true_type(), [&](int pos, const float (&d)[4], uint2 jp) {
      bool take[4];
#pragma unroll
      for (int h = 0; h < 4; h++) take[h] = __float_as_uint(d[h]) < ucut;
      // most groups of four are taken by no lane: skip them uniformly
      if (__any(take[0] | take[1] | take[2] | take[3])) {
        const int4 jj = CL ? int4{(int)(jp.x & 0xFFFFu), (int)(jp.x >> 16), (int)(jp.y & 0xFFFFu),
                                  (int)(jp.y >> 16)}
                           : cand_idx4(pos);
        const int j4[4] = {jj.x, jj.y, jj.z, jj.w};
#pragma unroll
        for (int h = 0; h < 4; h++) {
          // exec-masked: only the taking lanes store (few lanes of a wave)
          if (take[h]) {
            const bool lo = __float_as_uint(d[h]) < ulo;
            buf_s[(lo ? slot_lo : slot_cut) * kBlk + lane] = make_key_finite(d[h], j4[h]);
            slot_lo += lo ? 1 : 0;
            slot_cut += lo ? 0 : 1;
          }
        }
      }
    });
    // region sizes: S = lo_total below the cut bin, C = total - S in it;
    // rows past a lane's own count, up to the wave-wide maximum rounded to
    // four (the sweep reads four rows per wait: eight made this phase the
    // kernel's VGPR peak, 94 instead of 72), read as padding
    const int cnt_c = total - lo_total;
    auto wave_max_i = [&](int v) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
      return __builtin_amdgcn_readfirstlane(v);
    };
    const int smax = wave_max_i(lo_total), cmax = wave_max_i(cnt_c);
    const int spad = (smax + 3) & ~3, cpad = (cmax + 3) & ~3;
    for (int i = lo_total + wv; i < spad; i += NW) buf_s[i * kBlk + lane] = PCR_KEY_PAD;
    for (int i = cnt_c + wv; i < cpad; i += NW) buf_s[(cut0 + i) * kBlk + lane] = PCR_KEY_PAD;
    __syncthreads();
    PCR_STAMP(3);

    // 5. rank: wave wv holds the keys wv, wv + NW, ... of each region and
    //    counts, for each, the keys below it in one sweep of that region's
    //    rows; the sweep is compiled for a few key counts so that no compare
    //    is wasted on empty key slots and none needs a guard.  A below-cut
    //    key's rank is its rank in its region; a cut-bin key's is S + its
    //    rank in its region.
    constexpr int kEL = (KSEL + NW - 1) / NW;  // below-cut keys per wave (S < k <= KSEL)
    constexpr int kEC = CAP / NW;              // cut-bin keys per wave (C <= CAP - cut0)
    constexpr int kE = kEC > kEL ? kEC : kEL;
    // one register set for both regions (the below-cut keys are placed before
    // the cut bin's are loaded): the selection's VGPRs bound how many other
    // waves share its CUs
    kkey key[kE];
    int rank[kE];
    const int nel = (smax - wv + NW - 1) / NW;
    const int nec = (cmax - wv + NW - 1) / NW;
    // rows [r0, r0 + rpad) against the first NE keys, four rows per wait
    auto sweep = [&](auto ne_c, int r0, int rpad) __attribute__((always_inline)) {
      constexpr int NE = decltype(ne_c)::value;
      for (int j2 = r0; j2 < r0 + rpad; j2 += 4) {
        kkey o[4];
#pragma unroll
        for (int u = 0; u < 4; u++) o[u] = buf_s[(j2 + u) * kBlk + lane];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int e = 0; e < NE; e++) rank[e] += o[u] < key[e] ? 1 : 0;
      }
    };
    auto sweep_n = [&](int ne, int r0, int rpad, auto km_c) __attribute__((always_inline)) {
      constexpr int KM = decltype(km_c)::value;
      if (ne <= 0) return;
      if (ne <= 1)
        sweep(std::integral_constant<int, 1>(), r0, rpad);
      else if (ne <= 2)
        sweep(std::integral_constant<int, 2>(), r0, rpad);
      else if (ne <= 3 || KM <= 3)
        sweep(std::integral_constant<int, (KM < 3 ? KM : 3)>(), r0, rpad);
      else if (ne <= 4 || KM <= 4)
        sweep(std::integral_constant<int, (KM < 4 ? KM : 4)>(), r0, rpad);
      else if (ne <= 6 || KM <= 6)
        sweep(std::integral_constant<int, (KM < 6 ? KM : 6)>(), r0, rpad);
      else if (ne <= 8 || KM <= 8)
        sweep(std::integral_constant<int, (KM < 8 ? KM : 8)>(), r0, rpad);
      else
        sweep(std::integral_constant<int, KM>(), r0, rpad);
    };
    // below-cut region: ranks within it are final
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const int i = wv + e * NW;
      key[e] = (e < kEL && i < lo_total) ? buf_s[i * kBlk + lane] : PCR_KEY_PAD;
      rank[e] = 0;
    }
    sweep_n(nel, 0, spad, std::integral_constant<int, kEL>());
    __syncthreads();  // the region's ranking reads are done
    // placed in rows [0, S), which the cut-bin sweep does not read
#pragma unroll
    for (int e = 0; e < kEL; e++)
      if (wv + e * NW < lo_total) buf_s[rank[e] * kBlk + lane] = key[e];
    // cut-bin region: rank S + its rank within the region, kept when < k
    // (rows [S, k) are below cut0, so no sweep reads them)
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const int i = wv + e * NW;
      key[e] = (e < kEC && i < cnt_c) ? buf_s[(cut0 + i) * kBlk + lane] : PCR_KEY_PAD;
      rank[e] = 0;
    }
    sweep_n(nec, cut0, cpad, std::integral_constant<int, kEC>());
    PCR_STAMP(4);
#pragma unroll
    for (int e = 0; e < kEC; e++) {
      const int r = lo_total + rank[e];
      if (wv + e * NW < cnt_c && r < k) buf_s[r * kBlk + lane] = key[e];
    }
    __syncthreads();
    PCR_STAMP(5);
    if (sorted_emit == 2) {
      // the workgroup's 64 rows of kSkeyK keys are one contiguous range:
      // consecutive threads store consecutive keys (knn_emit_kernel
      // un-permutes them)
      kkey* rows = qs.skey + ((size_t)b * qs.npad + (size_t)qblk * kBlk) * kSkeyK;
      for (int e = threadIdx.x; e < kBlk * k; e += NW * kBlk) {
        const int q = e / k, sl = e - q * k;
        // nontemporal: 268 MB of key rows at c5, read once by the emit
        // (c5 KNN + PPF 2.12 -> 2.09 ms)
        __builtin_nontemporal_store(buf_s[sl * kBlk + q], &rows[(size_t)q * kSkeyK + sl]);
      }
      return;
    }
    if (!qlive) return;

    // output slots wv, wv + NW, ...
    constexpr int SPW = (KSEL + NW - 1) / NW;
    const int n = qs.n;
    int jn[SPW];
#pragma unroll
    for (int u = 0; u < SPW; u++) {
      const int sl = wv + u * NW;
      jn[u] = 0;
      if (sl < k) {
        const kkey x = buf_s[sl * kBlk + lane];
        const size_t o = ((size_t)b * k + sl) * n + qj;
        jn[u] = key_idx(x);
        if (dist) dist[o] = key_dist(x);
        if (sorted_emit)  // sorted query order: whole rows (see kSortedMaxN)
          qs.sidx[((size_t)b * kSortedK + sl) * qs.npad + (size_t)qblk * kBlk + lane] = jn[u];
        else
          idx[o] = jn[u];
      }
    }
    if (PPF) {
      const float* qo = qxyz + (size_t)b * 3 * n;
      const float* qnr = qnrm + (size_t)b * 3 * n;
      const float* cb = cxyz + (size_t)b * 3 * m;
      const float* nb = cnrm + (size_t)b * 3 * m;
      const float ox = qo[qj], oy = qo[qj + n], oz = qo[qj + 2 * n];
      const float cnx = qnr[qj], cny = qnr[qj + n], cnz = qnr[qj + 2 * n];
      float nbr[SPW][6];
#pragma unroll
      for (int u = 0; u < SPW; u++) {
        const int j = jn[u];
        nbr[u][0] = cb[j];
        nbr[u][1] = cb[j + m];
        nbr[u][2] = cb[j + 2 * m];
        nbr[u][3] = nb[j];
        nbr[u][4] = nb[j + m];
        nbr[u][5] = nb[j + 2 * m];
      }
#pragma unroll
      for (int u = 0; u < SPW; u++) {
        const int sl = wv + u * NW;
        if (sl < k) {
          float f[4];
          pcr_local_ppf(ox, oy, oz, cnx, cny, cnz, nbr[u][0], nbr[u][1], nbr[u][2], nbr[u][3],
                        nbr[u][4], nbr[u][5], relative, f);
#pragma unroll
          for (int ch = 0; ch < 4; ch++) ppf[(((size_t)b * 4 + ch) * k + sl) * n + qj] = f[ch];
        }
      }
    }
    PCR_STAMP(6);
    return;
  }

  // fallback: wave 0, reference insertion scan, list in LDS (rows 0..k-1)
  if (wv != 0) return;
  const kkey undef = make_key(PCR_KNN_UNDEF, 0);
  for (int s2 = 0; s2 < k; s2++) buf_s[s2 * kBlk + lane] = undef;
  kkey kth = undef;
  for (int blk = 0; blk < nblk; blk++) {
    // cached clouds read the candidates from LDS (broadcast reads)
    const float* bx = CL ? cand_s + blk * kBlk : cs.x + cbase + (size_t)blk * kBlk;
    const float* by = CL ? cand_s + CACHE + blk * kBlk : cs.y + cbase + (size_t)blk * kBlk;
    const float* bz = CL ? cand_s + 2 * CACHE + blk * kBlk : cs.z + cbase + (size_t)blk * kBlk;
    const int* bj = cs.j + cbase + (size_t)blk * kBlk;
    for (int t = 0; t < kBlk; t++) {
      const kkey x = make_key(cand_dist(qx, qy, qz, bx[t], by[t], bz[t]),
                              CL ? (int)cand_j[blk * kBlk + t] : bj[t]);
      if (x < kth) {
        int s2 = k - 1;
        while (s2 > 0) {
          const kkey p = buf_s[(s2 - 1) * kBlk + lane];
          if (p < x) break;
          buf_s[s2 * kBlk + lane] = p;
          s2--;
        }
        buf_s[s2 * kBlk + lane] = x;
        kth = buf_s[(k - 1) * kBlk + lane];
      }
    }
  }
  if (!qlive) return;
  if (sorted_emit == 2) {
    kkey* row = qs.skey + ((size_t)b * qs.npad + (size_t)qblk * kBlk + lane) * kSkeyK;
    for (int s2 = 0; s2 < k; s2++) row[s2] = buf_s[s2 * kBlk + lane];
    return;
  }
  const int n = qs.n;
  for (int s2 = 0; s2 < k; s2++) {
    const kkey x = buf_s[s2 * kBlk + lane];
    const size_t o = ((size_t)b * k + s2) * n + qj;
    if (dist) dist[o] = key_dist(x);
    if (sorted_emit)
      qs.sidx[((size_t)b * kSortedK + s2) * qs.npad + (size_t)qblk * kBlk + lane] = key_idx(x);
    else
      idx[o] = key_idx(x);
  }
  if (PPF) {
    const float* qo = qxyz + (size_t)b * 3 * n;
    const float* qnr = qnrm + (size_t)b * 3 * n;
    const float* cb = cxyz + (size_t)b * 3 * m;
    const float* nb = cnrm + (size_t)b * 3 * m;
    const float ox = qo[qj], oy = qo[qj + n], oz = qo[qj + 2 * n];
    const float cnx = qnr[qj], cny = qnr[qj + n], cnz = qnr[qj + 2 * n];
    for (int s2 = 0; s2 < k; s2++) {
      const int j = key_idx(buf_s[s2 * kBlk + lane]);
      float f[4];
      pcr_local_ppf(ox, oy, oz, cnx, cny, cnz, cb[j], cb[j + m], cb[j + 2 * m], nb[j],
                    nb[j + m], nb[j + 2 * m], relative, f);
#pragma unroll
      for (int ch = 0; ch < 4; ch++) ppf[(((size_t)b * 4 + ch) * k + s2) * n + qj] = f[ch];
    }
  }
}

// ---------------------------------------------------------------------------
// knn_wsel_kernel (round 5): the self-KNN selection of clouds of <= 64 R
// points, k <= 32, transposed -- one query per wave instruction, the cloud's
// candidates in the lanes.  Lane l holds the Morton-sorted candidates
// 64 r + l (r < R) in registers for the whole launch, so a query costs:
//
//  1. distances  its R distances per lane with the reference's FMA chain
//                (knn.cu:20-23; two candidates per packed instruction);
//  2. threshold  count(d <= t) over the wave is one v_cmp + s_bcnt1 per
//                register (the count is a ballot across the lanes, so no
//                per-pair atomic and no histogram).  t starts from the
//                previous query's threshold (Morton neighbours have similar
//                k-th distances) and moves by count ~ t^1.5 interpolation,
//                bracketed, until k <= count <= 64: 1.5 passes on average;
//  3. compact    the <= 64 keys with d <= t into one lane each (ballot +
//                mbcnt slots in the wave's LDS row);
//  4. sort       a 64-lane bitonic sort of 32-bit keys (d bits >> 5 << 6 |
//                slot): DPP / swizzle partners, min / max / select per stage.
//                Two keys whose truncated distances tie inside the first k
//                send the query to the exact 64-bit sort, as do
//  5. edge cases no t with k <= count <= 64 (exact duplicates, clusters):
//                the exact k-th distance by bisection of its float bits, the
//                tie at it broken by bisection of the original index, the
//                exactly k members compacted and sorted on 64-bit keys.
//
// Result: the k lexicographically smallest (d, original index) with d <
// 10000, unfilled slots index 0 -- the reference's insertion-sort result
// (knn.cu:24-46).  Written as neighbour ids in sorted query order (KnnSet::
// sidx rows, like knn_select_kernel's sorted_emit 1) through an LDS tile, so
// every store is a whole 256-byte row.
// Waves per workgroup (one 64-query block), W, and the queries a wave takes
// from the block's counter at a time, wsel_chunk<W>.  A launch of at most
// 4096 waves at W = 8 (c2: 32 clouds x 16 blocks) leaves 4 waves per SIMD:
// there W = 12 (the compiler then fits the kernel in 81 VGPRs instead of 91)
// taking one query at a time, c2 +1.7% (profiles/r06_ab_wsel_waves.log,
// r06_ab_wsel_chunk.log, r06_ab_wsel_pairs_waves.log; 10 waves -3%, 14 / 16
// spill SGPRs, -12%).  Larger launches (pairs: 256 clouds) keep W = 8 with
// two queries at a time: each wave stages the whole cloud in registers, and
// 12 waves cost pairs 9% (312-315k against 341-343k clouds/s).
template <int W>
constexpr int wsel_chunk() { return W == 8 ? 2 : 1; }
constexpr int kWselCap = 64;   // keys collected per query (one per lane)
constexpr int kWselTmax = 0x461C3FFF;  // bits of the largest float below 10000

// One compare-exchange stage of the sort below where the lower lanes of the
// pairs are the even lanes (m = 1) or lanes 0-1 of each quad (m = 2): the
// partner by DPP, folded into the compare and the select (2 VALU + 2 SALU):
// the borrow of partner - x (v_sub_co: VOPC has no DPP form on gfx950) is vcc
// = partner < x, flipped on the lanes that keep the minimum, then x = vcc ? x
// : partner.  s_nop 1: the previous stage's VALU wrote x, which this DPP
// reads (gfx9 needs 2 wait states).
#define PCR_WSEL_VCC_STAGE(NAME, CTRL, LOW)                                        \
  __device__ inline unsigned NAME(unsigned x) {                                    \
    unsigned t;                                                                    \
    asm volatile("s_nop 1\n\t"                                                     \
                 "v_sub_co_u32_dpp %1, vcc, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n\t" \
                 "s_xor_b32 vcc_lo, vcc_lo, " LOW "\n\t"                           \
                 "s_xor_b32 vcc_hi, vcc_hi, " LOW "\n\t"                           \
                 "v_cndmask_b32_dpp %0, %0, %0, vcc " CTRL " row_mask:0xf bank_mask:0xf" \
                 : "+v"(x), "=&v"(t)                                               \
                 :                                                                 \
                 : "vcc");                                                         \
    return x;                                                                      \
  }
PCR_WSEL_VCC_STAGE(wsel_x1, "quad_perm:[1,0,3,2]", "0x55555555")
PCR_WSEL_VCC_STAGE(wsel_x2, "quad_perm:[2,3,0,1]", "0x33333333")
PCR_WSEL_VCC_STAGE(wsel_m4, "quad_perm:[3,2,1,0]", "0x33333333")
#undef PCR_WSEL_VCC_STAGE
// Stages whose lower lanes are whole 4-lane banks of a row (m = 4, 8) or whole
// rows (m = 16, 32): the DPP bank / row masks pick the lanes, so the lower
// lanes write min(partner, x) and the upper lanes max(partner, x) into a new
// register with two masked VALU -- no VCC, no SALU.  LO / HI are the
// partner's DPP controls for the lower / upper lanes, MLO / MHI their masks.
#define PCR_WSEL_MINMAX_STAGE(NAME, LO, HI, MLO, MHI)                              \
  __device__ inline unsigned NAME(unsigned x) {                                    \
    unsigned a;                                                                    \
    asm volatile("s_nop 1\n\t"                                                     \
                 "v_min_u32_dpp %0, %1, %1 " LO " " MLO "\n\t"                     \
                 "v_max_u32_dpp %0, %1, %1 " HI " " MHI                            \
                 : "=&v"(a)                                                        \
                 : "v"(x));                                                        \
    return a;                                                                      \
  }
PCR_WSEL_MINMAX_STAGE(wsel_m8, "row_half_mirror", "row_half_mirror",
                      "row_mask:0xf bank_mask:0x5", "row_mask:0xf bank_mask:0xa")
PCR_WSEL_MINMAX_STAGE(wsel_m16, "row_mirror", "row_mirror",
                      "row_mask:0xf bank_mask:0x3", "row_mask:0xf bank_mask:0xc")
PCR_WSEL_MINMAX_STAGE(wsel_x4, "row_shl:4", "row_shr:4",
                      "row_mask:0xf bank_mask:0x5", "row_mask:0xf bank_mask:0xa")
PCR_WSEL_MINMAX_STAGE(wsel_x8, "row_shl:8", "row_shr:8",
                      "row_mask:0xf bank_mask:0x3", "row_mask:0xf bank_mask:0xc")
#undef PCR_WSEL_MINMAX_STAGE
// Cross-row partners (FETCH into %2): lane ^ 16 / lane ^ 32 from gfx950's
// v_permlane16_swap / v_permlane32_swap of a register with itself, the 32- and
// 64-lane mirrors from a row mirror plus those swaps; then the row-masked
// min / max (identity DPP: only its row mask matters).  No LDS round trip.
#define PCR_WSEL_ROW_STAGE(NAME, FETCH, RLO, RHI)                                  \
  __device__ inline unsigned NAME(unsigned x) {                                    \
    unsigned a, p;                                                                 \
    asm volatile("s_nop 1\n\t" FETCH                                               \
                 "s_nop 1\n\t"                                                     \
                 "v_min_u32_dpp %0, %1, %2 quad_perm:[0,1,2,3] row_mask:" RLO " bank_mask:0xf\n\t" \
                 "v_max_u32_dpp %0, %1, %2 quad_perm:[0,1,2,3] row_mask:" RHI " bank_mask:0xf" \
                 : "=&v"(a), "+v"(x), "=&v"(p)                                     \
                 :);                                                               \
    return a;                                                                      \
  }
PCR_WSEL_ROW_STAGE(wsel_x16,
                   "v_mov_b32_e32 %2, %1\n\t"
                   "s_nop 1\n\t"
                   "v_permlane16_swap_b32 %2, %2\n\t",
                   "0x5", "0xa")
PCR_WSEL_ROW_STAGE(wsel_m32,
                   "v_mov_b32_dpp %2, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
                   "s_nop 1\n\t"
                   "v_permlane16_swap_b32 %2, %2\n\t",
                   "0x5", "0xa")
PCR_WSEL_ROW_STAGE(wsel_m64,
                   "v_mov_b32_dpp %2, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
                   "s_nop 1\n\t"
                   "v_permlane16_swap_b32 %2, %2\n\t"
                   "s_nop 1\n\t"
                   "v_permlane32_swap_b32 %2, %2\n\t",
                   "0x3", "0xc")
#undef PCR_WSEL_ROW_STAGE

// ascending 64-lane bitonic sort ("mirror" form: the first stage of each
// merge compares i with its mirror i ^ (kk - 1), so every block sorts
// ascending and the lower lane of a pair always keeps the minimum)
__device__ inline unsigned wsel_sort64(unsigned x) {
  x = wsel_x1(x);
  x = wsel_m4(x);
  x = wsel_x1(x);
  x = wsel_m8(x);
  x = wsel_x2(x);
  x = wsel_x1(x);
  x = wsel_m16(x);
  x = wsel_x4(x);
  x = wsel_x2(x);
  x = wsel_x1(x);
  x = wsel_m32(x);
  x = wsel_x8(x);
  x = wsel_x4(x);
  x = wsel_x2(x);
  x = wsel_x1(x);
  x = wsel_m64(x);
  x = wsel_x16(x);
  x = wsel_x8(x);
  x = wsel_x4(x);
  x = wsel_x2(x);
  x = wsel_x1(x);
  // the caller's next DPP read of x follows a VALU write inside the asm above,
  // which the compiler's hazard tracking does not see
  asm volatile("s_nop 1");
  return x;
}

// the same on 64-bit keys (d bits << 32 | original index): exact, rare
__device__ inline unsigned long long wsel_sort64_exact(unsigned long long x, int lane) {
  for (int kk = 2; kk <= 64; kk <<= 1) {
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      const int m = jj == (kk >> 1) ? kk - 1 : jj;  // mirror first, then half-cleaners
      const unsigned long long p = shfl_xor_u64(x, m);
      const bool lower = (lane & jj) == 0;
      x = lower ? (x < p ? x : p) : (x < p ? p : x);
    }
  }
  return x;
}

// Appends the keys of the lanes in `m` (a ballot mask) to the wave's LDS
// rows at slots base, base + 1, ...: d bits to kd, index to kd + 256 bytes.
// exec = m for three VALU (the slot: mbcnt lo / hi; the address) and two
// ds_write, restored after: no per-lane condition is materialised.
__device__ inline void wsel_append(unsigned long long m, unsigned addr, unsigned d, int j) {
  unsigned t;
  unsigned long long save;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, %2\n\t"
      "v_mbcnt_lo_u32_b32 %0, %3, 0\n\t"
      "v_mbcnt_hi_u32_b32 %0, %4, %0\n\t"
      "v_lshl_add_u32 %0, %0, 2, %5\n\t"
      "ds_write_b32 %0, %6\n\t"
      "ds_write_b32 %0, %7 offset:256\n\t"
      "s_mov_b64 exec, %1"
      : "=&v"(t), "=&s"(save)
      : "s"(m), "s"((unsigned)m), "s"((unsigned)(m >> 32)), "s"(addr), "v"(d), "v"(j)
      : "memory");
}

template <int R, int W>
__global__ __launch_bounds__(W * 64) void knn_wsel_kernel(KnnSet s, int k) {
  constexpr int kWselWaves = W;
  constexpr int kWselChunk = wsel_chunk<W>();
  // [wave][0][slot] collected d bits, [wave][1][slot] their sorted positions
  // (256 bytes apart: wsel_append's ds_write offset)
  __shared__ unsigned kbuf_s[kWselWaves][2][kWselCap];
  __shared__ int tile_s[kBlk][kSortedK + 1];  // output ids [query][slot] (padded: no bank conflicts)
  __shared__ int qnext_s;                     // the next chunk of the block's queries
  __shared__ int cj_s[R * kBlk];              // original index of each sorted position
  static_assert(sizeof(kbuf_s[0][0]) == 256, "wsel_append's offset");
  const int b = blockIdx.y, qblk = blockIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t cb = (size_t)b * s.npad;
  const int nr = s.npad / kBlk;  // candidate registers in use (<= R)
  typedef float pf2v __attribute__((ext_vector_type(2)));
  // the whole cloud, one candidate per lane and register (NaN padding); the
  // candidates' original indices in LDS (cj_s[p], p = 64 r + lane: the
  // compaction stores positions, the output looks the index up)
  pf2v cx[R / 2], cy[R / 2], cz[R / 2];
  for (int i = threadIdx.x; i < R * kBlk; i += kWselWaves * kBlk)
    cj_s[i] = i < s.npad ? s.j[cb + i] : -1;
#pragma unroll
  for (int h = 0; h < R / 2; h++) {
    float v[2][3];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      // unconditional loads (a register past the cloud re-reads its last
      // block, then reads as NaN / -1): no branch, so all are in flight at once
      const int r = 2 * h + e;
      const bool ok = r < nr;
      const size_t p = cb + (size_t)(ok ? r : nr - 1) * kBlk + lane;
      const float x = s.x[p], y = s.y[p], z = s.z[p];
      v[e][0] = ok ? x : __builtin_nanf("");
      v[e][1] = ok ? y : __builtin_nanf("");
      v[e][2] = ok ? z : __builtin_nanf("");
    }
    cx[h] = pf2v{v[0][0], v[1][0]};
    cy[h] = pf2v{v[0][1], v[1][1]};
    cz[h] = pf2v{v[0][2], v[1][2]};
  }
  // the block's 64 queries, one per lane (every wave holds all of them: the
  // waves take chunks of kWselChunk consecutive queries from an LDS counter,
  // so a wave that drew expensive queries -- outliers, extra passes -- takes
  // fewer chunks and the workgroup ends with its mean, not its slowest wave)
  const size_t pq = cb + (size_t)qblk * kBlk + lane;
  const float qxl = s.x[pq], qyl = s.y[pq], qzl = s.z[pq];
  const int qjl = s.j[pq];
  if (threadIdx.x == 0) qnext_s = 0;
  __syncthreads();
  auto grab = [&]() {
    int v = 0;
    if (lane == 0)
      v = __hip_atomic_fetch_add(&qnext_s, kWselChunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return v;
  };
  int q0 = __builtin_amdgcn_readfirstlane(grab());
  // first guess: the largest distance from the wave's first query to its own
  // block's box (>= the k-th when the block holds k points), else 10000-
  int tb = kWselTmax;
  if (q0 < kBlk) {
    const float* bx = s.box + ((size_t)b * s.nblk + qblk) * 8;
    const float qx = readlane_f(qxl, q0), qy = readlane_f(qyl, q0), qz = readlane_f(qzl, q0);
    if (min(kBlk, s.n - qblk * kBlk) >= k) {
      const float u = box_ub(qx, qy, qz, bx);
      if (u < PCR_KNN_UNDEF) tb = (int)__float_as_uint(u);
    }
  }
  unsigned* kd = kbuf_s[wv][0];
  int* kj = (int*)kbuf_s[wv][1];
  const unsigned kd_addr =  // LDS byte address of the wave's rows
      (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned*)kd);
  const float tgt = 0.5f * (float)(k + kWselCap);
#pragma unroll 1
  for (int qi = q0; qi < kBlk;) {
    const int qj = __builtin_amdgcn_readlane(qjl, qi);
    if (qj < 0) {
      if (lane < kSortedK) tile_s[qi][lane] = 0;
      if (++qi % kWselChunk == 0) qi = __builtin_amdgcn_readfirstlane(grab());
      continue;
    }
    const float qx = readlane_f(qxl, qi), qy = readlane_f(qyl, qi), qz = readlane_f(qzl, qi);
    const pf2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
    // 1. distances, knn.cu:20-23's chain
    unsigned db[R];
#pragma unroll
    for (int h = 0; h < R / 2; h++) {
      const pf2v a = qx2 - cx[h], bq = qy2 - cy[h], c = qz2 - cz[h];
      pf2v d = a * a;
      d = __builtin_elementwise_fma(bq, bq, d);
      d = __builtin_elementwise_fma(c, c, d);
      db[2 * h] = __float_as_uint(d[0]);
      db[2 * h + 1] = __float_as_uint(d[1]);
    }
    // 2. threshold: count(d <= t) by ballots (NaN bits compare above every t)
    // the last pass's ballots are kept for the compaction when they fit in
    // SGPRs (R = 16: 32 of them); R = 32 ballots again there
    constexpr bool kKeep = R <= 16;
    unsigned long long msk[kKeep ? R : 1];
    auto count_le = [&](int bits) {
      // four running popcount sums: a dependency chain a quarter as long
      int pc[4] = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < R; r++) {
        const unsigned long long m = __ballot(db[r] <= (unsigned)bits);
        if (kKeep) msk[kKeep ? r : 0] = m;
        pc[r & 3] += __popcll(m);
      }
      return (pc[0] + pc[1]) + (pc[2] + pc[3]);
    };
    int lo = -1, hi = 0x7F800000, cnt_lo = 0, cnt = 0;
    bool exact = false;
#pragma unroll 1
    for (int pass = 0;; pass++) {
      cnt = count_le(tb);
      if (cnt >= k && cnt <= kWselCap) break;
      if (cnt < k) {
        lo = tb;
        cnt_lo = cnt;
        if (tb >= kWselTmax) break;  // fewer than k candidates below 10000: all of them
      } else {
        hi = tb;
      }
      if (hi - lo <= 1) {  // more than 64 - cnt_lo keys tie at distance bits hi
        exact = true;
        break;
      }
      int nb;
      if (pass < 3) {
        // count ~ t^1.5 near the k-th distance (smooth clouds: ~1.6 passes)
        // (raw v_log / v_exp: any estimate is correct here, the bracket
        // below keeps it inside (lo, hi); the library forms add range fixups)
        const float f = __uint_as_float((unsigned)tb) *
                        __builtin_amdgcn_exp2f(0.6666667f * __builtin_amdgcn_logf(
                                                                tgt * __builtin_amdgcn_rcpf((float)max(cnt, 1))));
        nb = f < 1e30f ? (int)__float_as_uint(f) : kWselTmax;
      } else {
        // steep counts (an outlier facing the bulk): bisect the bracket's bits
        nb = lo + ((hi - lo) >> 1);
      }
      nb = min(nb, kWselTmax);
      if (nb <= lo || nb >= hi) nb = lo + ((hi - lo) >> 1);
      tb = __builtin_amdgcn_readfirstlane(nb);
    }
    int ntake;
    if (!exact) {
      // 3. compact the cnt <= 64 keys with d <= t (the last pass's ballots)
      unsigned addr = kd_addr;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const unsigned long long m = kKeep ? msk[kKeep ? r : 0] : __ballot(db[r] <= (unsigned)tb);
        if (m != 0ull) {
          wsel_append(m, addr, db[r], 64 * r + pcr_opaque(lane));
          addr += 4u * (unsigned)__popcll(m);
        }
      }
      ntake = cnt;
    } else {
      // 5. ties: every key below distance bits hi (cnt_lo < k of them), then
      // the need = k - cnt_lo smallest indices among those at exactly hi
      const int need = k - cnt_lo;
      // (rare: the indices are read from LDS where used, no registers held)
      auto cj = [&](int r) { return cj_s[64 * r + lane]; };
      int jl = -1, jh = s.n - 1;
#pragma unroll 1
      while (jh - jl > 1) {
        const int jm = jl + ((jh - jl) >> 1);
        int c = 0;
#pragma unroll
        for (int r = 0; r < R; r++) c += __popcll(__ballot(db[r] == (unsigned)hi && cj(r) <= jm));
        if (c >= need) jh = jm;
        else jl = jm;
      }
      unsigned addr = kd_addr;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const unsigned long long m =
            __ballot(db[r] < (unsigned)hi || (db[r] == (unsigned)hi && cj(r) <= jh));
        if (m != 0ull) {
          wsel_append(m, addr, db[r], 64 * r + pcr_opaque(lane));
          addr += 4u * (unsigned)__popcll(m);
        }
      }
      ntake = k;
    }
    // 4. sort 31-bit keys: d bits >> 6 (25 bits: d < 10000) and the slot as payload
    const unsigned dl = lane < ntake ? kd[lane] : 0xFFFFFFFFu;
    unsigned key = lane < ntake ? ((dl >> 6) << 6) | (unsigned)lane : 0x7FFFFFFFu;
    key = wsel_sort64(key);
    // a truncated-distance tie among the first k (or at the k-th) needs the
    // exact order (lane i sees lane i + 1: DPP wave_shl:1)
    const unsigned nxt = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x130, 0xF, 0xF, false);
    const bool tie = lane < k && lane + 1 < ntake && (key >> 6) == (nxt >> 6);
    const bool slow = __any(tie);
    if (!slow) {
      const int jo = lane < ntake ? cj_s[kj[key & 63u]] : 0;
      if (lane < k) tile_s[qi][lane] = jo;
    } else {
      unsigned long long skey = ~0ull;
      if (lane < ntake) skey = ((unsigned long long)kd[lane] << 32) | (unsigned)cj_s[kj[lane]];
      skey = wsel_sort64_exact(skey, lane);
      if (lane < k) tile_s[qi][lane] = lane < ntake ? (int)(unsigned)(skey & 0xFFFFFFFFull) : 0;
    }
    // the rows are read before the next query's appends rewrite them (LDS
    // operations of a wave complete in order; this keeps the compiler's order)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (++qi % kWselChunk == 0) qi = __builtin_amdgcn_readfirstlane(grab());
  }
  __syncthreads();
  for (int sl = wv; sl < k; sl += kWselWaves)
    s.sidx[((size_t)b * kSortedK + sl) * s.npad + (size_t)qblk * kBlk + lane] = tile_s[lane][sl];
}

// Un-permutes the selection's sorted-order keys (qs.skey, sorted_emit 2)
// into the reference's [b][k][n] outputs (knn/knn.cu:40-47 layout) and
// computes the local PPF of every (query, slot) on the way
// (models/pvcnn_classify.py:252-269, the same pcr_local_ppf call as the
// selection's own epilogue).  One wave per 64 consecutive original queries
// and 16 slots (16 contiguous keys of each query's row: one 128-byte line
// per lane); every output store is a whole 256-byte row.
// XCD-aware: the dispatcher deals workgroups round-robin over the 8 XCDs, so
// work unit (blockIdx.x % 8) * (grid / 8) + blockIdx.x / 8 keeps a run of
// consecutive query blocks -- one cloud's neighbour gathers -- in one L2.
template <bool PPF>
__global__ __launch_bounds__(256) void knn_emit_kernel(KnnSet qs, int k, int nqb, float* dist,
                                                       int* idx, const float* __restrict__ qxyz,
                                                       const float* __restrict__ qnrm,
                                                       const float* __restrict__ crec, int m,
                                                       int relative, float* ppf) {
  constexpr int kChunk = kSkeyK / 4;  // slots per wave
  constexpr int kG = 4;               // slots whose neighbours are gathered together
  const int total = gridDim.x;
  int u = blockIdx.x;
  if ((total & 7) == 0) u = (u & 7) * (total >> 3) + (u >> 3);
  const int b = u / nqb, qb = u - b * nqb;
  const int n = qs.n;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qj = qb * kBlk + lane;
  const int s0 = wv * kChunk;
  if (qj >= n || s0 >= k) return;  // no barrier below
  const int ns = min(k - s0, kChunk);
  const int p = qs.inv[(size_t)b * n + qj];
  // the wave's 16 keys of the query's row at once (one 128-byte line per
  // lane; the row always holds kSkeyK keys, so no guard): each line is
  // fetched once, not once per slot
  const double2* row = (const double2*)(qs.skey + ((size_t)b * qs.npad + p) * kSkeyK + s0);
  kkey key[kChunk];
#pragma unroll
  for (int i = 0; i < kChunk / 2; i++) {
    const double2 v = row[i];
    key[i * 2] = v.x;
    key[i * 2 + 1] = v.y;
  }
  float ox = 0.0f, oy = 0.0f, oz = 0.0f, cnx = 0.0f, cny = 0.0f, cnz = 0.0f;
  // a neighbour's point and normal as one 32-byte record (two dwordx4): one
  // line per gather instead of six
  const float4* rb = (const float4*)(crec + (size_t)b * m * 8);
  if (PPF) {
    const float* qo = qxyz + (size_t)b * 3 * n;
    const float* qnr = qnrm + (size_t)b * 3 * n;
    ox = qo[qj];
    oy = qo[qj + n];
    oz = qo[qj + 2 * n];
    cnx = qnr[qj];
    cny = qnr[qj + n];
    cnz = qnr[qj + 2 * n];
  }
#pragma unroll
  for (int g = 0; g < kChunk; g += kG) {
    if (g >= ns) break;
    float nbr[kG][6];
#pragma unroll
    for (int t = 0; t < kG; t++) {
      const int j = g + t < ns ? key_idx(key[g + t]) : 0;
      if (PPF) {
        const float4 r0 = rb[2 * (size_t)j], r1 = rb[2 * (size_t)j + 1];
        nbr[t][0] = r0.x;
        nbr[t][1] = r0.y;
        nbr[t][2] = r0.z;
        nbr[t][3] = r0.w;
        nbr[t][4] = r1.x;
        nbr[t][5] = r1.y;
      }
    }
#pragma unroll
    for (int t = 0; t < kG; t++) {
      if (g + t >= ns) break;
      const int sl = s0 + g + t;
      const size_t o = ((size_t)b * k + sl) * n + qj;
      // streamed outputs (far larger than the L2 / MALL): nontemporal stores
      // (c5 KNN + PPF 2.20 -> 2.12 ms)
#define PCR_EST(p, v) __builtin_nontemporal_store((v), &(p))
      if (idx) PCR_EST(idx[o], key_idx(key[g + t]));
      if (dist) PCR_EST(dist[o], key_dist(key[g + t]));
      if (PPF) {
        float f[4];
        pcr_local_ppf(ox, oy, oz, cnx, cny, cnz, nbr[t][0], nbr[t][1], nbr[t][2], nbr[t][3],
                      nbr[t][4], nbr[t][5], relative, f);
#pragma unroll
        for (int ch = 0; ch < 4; ch++) PCR_EST(ppf[(((size_t)b * 4 + ch) * k + sl) * n + qj], f[ch]);
      }
    }
  }
}

// [b][3][m] points + normals -> [b][m][8] records (x y z nx ny nz 0 0)
__global__ __launch_bounds__(256) void knn_pack_rec_kernel(const float* __restrict__ xyz,
                                                           const float* __restrict__ nrm, int m,
                                                           float* __restrict__ rec) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= m) return;
  const float* P = xyz + (size_t)b * 3 * m;
  const float* N = nrm + (size_t)b * 3 * m;
  float4* r = (float4*)(rec + ((size_t)b * m + i) * 8);
  r[0] = float4{P[i], P[i + m], P[i + 2 * (size_t)m], N[i]};
  r[1] = float4{N[i + m], N[i + 2 * (size_t)m], 0.0f, 0.0f};
}

template <bool PPF>
static void launch_emit(const KnnSet& qs, const KnnSet& cs, int b, int k, float* dist, int* idx,
                        const float* qxyz, const float* qnrm, const float* cxyz,
                        const float* cnrm, int relative, float* ppf, hipStream_t st) {
  const int nqb = ceil_div(qs.n, kBlk);
  // the candidates' records, in the candidate set's workspace
  if (PPF)
    hipLaunchKernelGGL(knn_pack_rec_kernel, dim3(ceil_div(cs.n, 256), b), dim3(256), 0, st, cxyz,
                       cnrm, cs.n, cs.rec);
  hipLaunchKernelGGL((knn_emit_kernel<PPF>), dim3(nqb * b), dim3(256), 0, st, qs, k, nqb, dist,
                     idx, qxyz, qnrm, cs.rec, cs.n, relative, ppf);
}

template <int NW, bool PPF, int CAP = kCap, int KSEL = kSelMaxK>
static void launch_select(const KnnSet& qs, const KnnSet& cs, int b, int k, float* dist,
                          int* idx, const float* qxyz, const float* qnrm, const float* cxyz,
                          const float* cnrm, int relative, float* ppf, hipStream_t st,
                          int sorted_emit = 0) {
  // a wave sees ceil(nblk / NW) * 64 candidates: byte fields when that fits
  PCR_PRIO_INIT();
  const int per_wave = ceil_div(cs.nblk, NW) * kBlk;
  const dim3 grid(qs.nblk, b), blk(NW * 64);
#define PCR_SEL(CBV, CLV, CACHEV)                                                             \
  hipLaunchKernelGGL((knn_select_kernel<NW, CBV, CLV, PPF, CAP, KSEL, CACHEV>), grid, blk, 0, st, \
                     qs, cs, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf,              \
                     sorted_emit)
  if constexpr (CAP == kCap) {
    // c3 clouds (2048 points): 32 KB of candidates in LDS, two workgroups per CU
    if (cs.npad > kSelCache && cs.npad <= 2 * kSelCache) {
      PCR_SEL(16, true, 2 * kSelCache);
      return;
    }
  }
  if (per_wave <= 255 && cs.npad <= kSelCache)
    PCR_SEL(8, true, kSelCache);
  else if (per_wave <= 255)
    PCR_SEL(8, false, kSelCache);
  else
    PCR_SEL(16, false, kSelCache);
#undef PCR_SEL
}

size_t knn_ws_size(int b, int n, int m) {
  size_t off = knn_set_layout(b, n, nullptr, nullptr, 0);
  return knn_set_layout(b, m, nullptr, nullptr, off);
}

static int next_pow2i(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static void launch_sort(const float* pts, int b, int n, const KnnSet& s, hipStream_t st) {
  PCR_PRIO_INIT();
  if (n > kKnnMaxSortN) {
    hipLaunchKernelGGL(knn_big_frame_kernel, dim3(b), dim3(kSortBlock), 0, st, pts, n, s);
    hipLaunchKernelGGL(knn_big_count_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0, st, pts, n,
                       s);
    hipLaunchKernelGGL(knn_big_scan_kernel, dim3(b), dim3(kSortBlock), 0, st, s);
    hipLaunchKernelGGL(knn_big_scatter_kernel, dim3(ceil_div(s.npad, 256), b), dim3(256), 0, st,
                       pts, n, s);
    hipLaunchKernelGGL(knn_big_boxes_kernel, dim3(ceil_div(s.nblk, 4), b), dim3(256), 0, st, s);
    return;
  }
  // clouds of <= 1024 points: 256 threads (four points each), so the sort
  // fits on a CU beside the other stream's grid kernel
  const size_t smem = 4096 * 4 + (size_t)n * 16;  // hist | order | sorted x y z
  if (n <= kSmallSortN) {
    const int npad_sort = next_pow2i(n < kSmallSortThreads ? kSmallSortThreads : n);
    allow_big_lds(knn_sort_kernel<kSmallSortThreads>, smem);
    hipLaunchKernelGGL((knn_sort_kernel<kSmallSortThreads>), dim3(b), dim3(kSmallSortThreads),
                       smem, st, pts, n, npad_sort, s);
  } else {
    const int npad_sort = next_pow2i(n < kSortBlock ? kSortBlock : n);
    allow_big_lds(knn_sort_kernel<kSortBlock>, smem);
    hipLaunchKernelGGL((knn_sort_kernel<kSortBlock>), dim3(b), dim3(kSortBlock), smem, st, pts,
                       n, npad_sort, s);
  }
}

template <int KM, bool PPF>
static void launch_block_k(const KnnSet& qs, const KnnSet& cs, int b, int k, float* dist,
                           int* idx, const float* qxyz, const float* qnrm, const float* cxyz,
                           const float* cnrm, int relative, float* ppf, hipStream_t st) {
  dim3 grid(ceil_div(qs.nblk, KnnNW<KM>::wg / KnnNW<KM>::value), b);
  hipLaunchKernelGGL((knn_block_kernel<KM, PPF>), grid, dim3(KnnNW<KM>::wg * 64), 0, st, qs, cs, k,
                     dist, idx,
                     qxyz, qnrm, cxyz, cnrm, relative, ppf);
}

template <bool PPF>
static pcr_status launch_block(const KnnSet& qs, const KnnSet& cs, int b, int k, float* dist,
                               int* idx, const float* qxyz, const float* qnrm, const float* cxyz,
                               const float* cnrm, int relative, float* ppf, hipStream_t st,
                               int sorted_emit = 0) {
  const bool sel = k <= kSelMaxK || (k <= kSelMaxK64 && cs.npad > kSelCache);
  if (sel && sorted_emit == 0 && qs.skey != nullptr) {
    // queries past kSortedMaxN: keys in sorted query order, then un-permuted
    if (k <= kSelMaxK)
      launch_select<8, false>(qs, cs, b, k, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                              0, nullptr, st, 2);
    else
      launch_select<8, false, kCap64, kSelMaxK64>(qs, cs, b, k, nullptr, nullptr, nullptr,
                                                  nullptr, nullptr, nullptr, 0, nullptr, st, 2);
    launch_emit<PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st);
    return PCR_OK;
  }
  if (k <= kSelMaxK) {
    launch_select<8, PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st,
                          sorted_emit);
  } else if (k <= kSelMaxK64 && cs.npad > kSelCache) {
    // large clouds (BASELINE c5, k = 64): the pruned threshold selection with
    // room for 2.75 k collected keys per query
    launch_select<8, PPF, kCap64, kSelMaxK64>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm,
                                              relative, ppf, st);
  } else if (k <= 16)
    launch_block_k<16, PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st);
  else if (k <= 32)
    launch_block_k<32, PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st);
  else if (k <= 64)
    launch_block_k<64, PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st);
  else if (k <= 128)
    launch_block_k<128, PPF>(qs, cs, b, k, dist, idx, qxyz, qnrm, cxyz, cnrm, relative, ppf, st);
  else
    return PCR_ERR_UNSUPPORTED;
  return PCR_OK;
}

// Returns PCR_ERR_UNSUPPORTED (nothing launched) when the spatial path does
// not apply; the caller then uses the brute-force kernels.
pcr_status knn_spatial(const float* xyz1, const float* xyz2, int b, int n, int m, int k,
                       float* dist1, int* idx1, float* dist2, int* idx2, const float* nrm1,
                       const float* nrm2, int relative, float* ppf1, void* ws, size_t ws_bytes,
                       bool self, hipStream_t st, int stages) {
  if (ws == nullptr || n > kKnnMaxN || m > kKnnMaxN || n < 1 || m < 1 || k > 128)
    return PCR_ERR_UNSUPPORTED;
  if (ws_bytes < knn_ws_size(b, n, m)) return PCR_ERR_UNSUPPORTED;
  KnnSet s1, s2;
  size_t off = knn_set_layout(b, n, &s1, (char*)ws, 0);
  knn_set_layout(b, m, &s2, (char*)ws, off);
  if (stages & 1) {
    launch_sort(xyz1, b, n, s1, st);
    if (!self) launch_sort(xyz2, b, m, s2, st);
  }
  if (!(stages & 2)) return PCR_OK;
  const KnnSet& c1 = self ? s1 : s2;
  pcr_status rc;
  if (stages & 4) {
    // selection only, neighbour ids in sorted query order into s1.sidx (the
    // cached selection, k <= kSortedK); the caller's PPF launch un-permutes
    if (!self || ppf1 || dist1 || idx2 || k > kSortedK || k > kSelMaxK || s1.sidx == nullptr ||
        s1.npad > 2 * kSelCache)
      return PCR_ERR_UNSUPPORTED;
    // clouds of <= 1024 points: the transposed selection (c2: 31.0 us alone
    // against 32.8 for knn_select_kernel).  At 2048 points its R = 32
    // registers per coordinate leave 2 waves per SIMD and it lost (928 us
    // against 600 at c3), so those keep the per-lane kernel.
    if (s1.npad <= 16 * kBlk) {
      if ((size_t)s1.nblk * b * 8 <= 4096)
        hipLaunchKernelGGL((knn_wsel_kernel<16, 12>), dim3(s1.nblk, b), dim3(12 * 64), 0, st, s1,
                           k);
      else
        hipLaunchKernelGGL((knn_wsel_kernel<16, 8>), dim3(s1.nblk, b), dim3(8 * 64), 0, st, s1,
                           k);
      return PCR_OK;
    }
    return launch_block<false>(s1, c1, b, k, nullptr, idx1, nullptr, nullptr, nullptr, nullptr,
                               0, nullptr, st, 1);
  }
  if (ppf1)
    rc = launch_block<true>(s1, c1, b, k, dist1, idx1, xyz1, nrm1, xyz2, nrm2, relative, ppf1, st);
  else
    rc = launch_block<false>(s1, c1, b, k, dist1, idx1, nullptr, nullptr, nullptr, nullptr, 0,
                             nullptr, st);
  if (rc != PCR_OK) return rc;
  if (idx2) rc = launch_block<false>(c1, s1, b, k, dist2, idx2, nullptr, nullptr, nullptr, nullptr,
                                     0, nullptr, st);
  return rc;
}

// the sorted-order outputs of a self KNN workspace (knn_spatial stage 4)
bool knn_sorted_views(void* ws, int b, int n, const int** sidx, const int** inv, int* npad) {
  KnnSet s;
  knn_set_layout(b, n, &s, (char*)ws, 0);
  *sidx = s.sidx;
  *inv = s.inv;
  *npad = s.npad;
  return s.sidx != nullptr;
}

}  // namespace pcr

extern "C" size_t pcr_knn_workspace_size(int b, int n, int m) {
  if (b <= 0 || n <= 0 || m <= 0) return 256;
  return pcr::knn_ws_size(b, n, m);
}

