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

// knn_spatial.hip: Morton-sorted exact KNN.  Returns PCR_ERR_UNSUPPORTED
// without launching anything when it does not apply.  stages: 1 = sort the
// point sets into the workspace, 2 = select from an already sorted workspace,
// 3 = both.
pcr_status knn_spatial(const float* xyz1, const float* xyz2, int b, int n, int m, int k,
                       float* dist1, int* idx1, float* dist2, int* idx2, const float* nrm1,
                       const float* nrm2, int relative, float* ppf1, void* ws, size_t ws_bytes,
                       bool self, hipStream_t st, int stages = 3);
// stage 4 (with 2): the selection writes its neighbour ids in sorted query
// order into the workspace (k <= 32, clouds of <= 2048 points); these are the
// views of that output and of the sort's inverse permutation
constexpr int kKnnSortedK = 32;
bool knn_sorted_views(void* ws, int b, int n, const int** sidx, const int** inv, int* npad);

// ---------------------------------------------------------------- device
constexpr int kWave = 64;

// Diagnostic phase stamps (separate build, -DPCR_DIAG, lib/libpcr_amd_diag.so):
// lane 0 of wave 0 of workgroup g records s_memtime at phase p into
// pcr_diag_stamps[g][p]; read back with pcr_diag_read().  Compiled out of the
// product library.
#ifdef PCR_DIAG
static __device__ unsigned long long pcr_diag_stamps[1024][16];  // one copy per TU
#define PCR_DIAG_READER(name)                                                       \
  extern "C" int name(unsigned long long* host) {                                  \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pcr::pcr_diag_stamps), sizeof(pcr::pcr_diag_stamps)); \
  }
#define PCR_WG_LINEAR (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z))
#define PCR_STAMP(p)                                                              \
  do {                                                                            \
    if (threadIdx.x == 0 && PCR_WG_LINEAR < 1024)                                 \
      pcr_diag_stamps[PCR_WG_LINEAR][p] = __builtin_amdgcn_s_memtime();           \
  } while (0)
#else
#define PCR_STAMP(p) \
  do {               \
  } while (0)
#endif

// Experiment knobs (launch shapes, schedule variants) are read from the
// environment only in the diagnostic build; the product library compiles the
// default in, so no environment variable can change what a timed run does.
#ifdef PCR_DIAG
#define PCR_KNOB(name, dflt) (getenv(name) ? atoi(getenv(name)) : (dflt))
#else
#define PCR_KNOB(name, dflt) (dflt)
#endif

// Issue priority of the latency-bound per-cloud kernels (prep, Morton sort):
// they share CUs with the other stream's throughput kernels, whose waves
// would otherwise take most issue slots and stretch them several-fold.
__device__ inline void latency_kernel_priority() { __builtin_amdgcn_s_setprio(3); }

// Diagnostic builds: per-kernel issue priorities from the environment
// (PCR_PRIO_<slot>=0..3, slot 0 sort, 1 select, 2 PPF, 3 prep, 4 means,
// 5 grid stream; -1 = the product's choice).  Each translation unit keeps its
// own copy of the table and loads it before its first launch.
#ifdef PCR_DIAG
static __device__ int pcr_prio_tab[8];
static inline void diag_prio_init() {
  static bool done = false;
  if (done) return;
  done = true;
  int t[8];
  char name[32];
  for (int i = 0; i < 8; i++) {
    snprintf(name, sizeof(name), "PCR_PRIO_%d", i);
    t[i] = getenv(name) ? atoi(getenv(name)) : -1;
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pcr_prio_tab), t, sizeof(t));
}
// returns true when the environment overrides this slot's priority
__device__ inline bool diag_prio(int slot) {
  const int p = __builtin_amdgcn_readfirstlane(pcr_prio_tab[slot]);
  if (p < 0) return false;
  if (p == 0) __builtin_amdgcn_s_setprio(0);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(3);
  return true;
}
#define PCR_PRIO_INIT() diag_prio_init()
#define PCR_PRIO(slot) diag_prio(slot)
#else
#define PCR_PRIO_INIT() \
  do {                  \
  } while (0)
#define PCR_PRIO(slot) false
#endif

// Workgroup barrier with LDS-scope fences.  On this toolchain (ROCm 7.2,
// gfx950) it still compiles to s_waitcnt vmcnt(0) lgkmcnt(0) before the
// s_barrier, exactly like __syncthreads(): every outstanding global load and
// store of the wave is waited for.  Where a kernel keeps global prefetches or
// stores in flight across a barrier it uses lds_only_barrier() below.
__device__ inline void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Workgroup barrier that waits only for this wave's LDS operations
// (s_waitcnt lgkmcnt(0); s_barrier; vmcnt and expcnt at their maxima, gfx9
// encoding): outstanding global loads, stores and LDS-DMA transfers stay in
// flight.  Only for data exchanged through LDS; an LDS-DMA target must be
// waited for with vmcnt by the issuing wave before the barrier.  The two
// builtins are IntrNoMem in LLVM, so on their own they do not stop IR passes
// from moving or forwarding LDS accesses across them: the signal fences are
// compiler-only barriers (they emit no instruction and no vmcnt wait).
__device__ inline void lds_only_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

typedef __attribute__((address_space(3))) void* lds_void_p;
typedef __attribute__((address_space(1))) void* gbl_void_p;

// s_waitcnt vmcnt(N) only (gfx9 encoding: expcnt / lgkmcnt at their maxima)
template <int N>
__device__ inline void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // compiler-only (the builtin is IntrNoMem)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Workgroup copy of `nbytes` (a multiple of V) from global memory straight
// into LDS by LDS-DMA (global_load_lds_dword / _dwordx4, V = 4 / 16 bytes per
// lane): the waves of the workgroup take pieces of 64 V bytes in turn and
// issue them all without waiting, so the whole copy is one round trip, and no
// staging registers are held.  Lanes of the last piece past the end re-read
// the last V bytes (in bounds) into the destination's tail, which must be
// padded to a whole piece (lds_dma_pad).  The caller waits with
// wait_vmcnt<0>() before the barrier that publishes the data.
__host__ __device__ inline int lds_dma_pad(int nbytes, int v) {
  return (nbytes + 64 * v - 1) / (64 * v) * (64 * v);
}
template <int V>
__device__ inline void lds_dma_copy(void* lds_dst, const void* gsrc, int nbytes) {
  static_assert(V == 4 || V == 16, "LDS-DMA width");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int np = (nbytes + 64 * V - 1) / (64 * V);
  for (int p = wv; p < np; p += nw) {
    const int off = min(p * 64 * V + lane * V, nbytes - V);
    const gbl_void_p src = (gbl_void_p)((const char*)gsrc + off);
    const lds_void_p dst = (lds_void_p)((char*)lds_dst + p * 64 * V);
    if constexpr (V == 16)
      __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds(src, dst, 4, 0, 0);
  }
}

// Inclusive block-wide scan of one int per thread (blockDim.x threads,
// multiple of 64, <= 1024).  `smem` needs blockDim.x/64 + 1 ints.  Its
// barriers order LDS only (lds_barrier).
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
  lds_barrier();
  if (wid == 0) {
    int w = (lane < nw) ? smem[lane] : 0;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      int t = __shfl_up(w, off, kWave);
      if (lane >= off) w += t;
    }
    if (lane < nw) smem[lane] = w;
  }
  lds_barrier();
  int base = (wid > 0) ? smem[wid - 1] : 0;
  lds_barrier();
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

// Block-wide sorts: kSortBlock threads, up to kMaxE keys per thread.
constexpr int kSortBlock = 1024;
constexpr int kMaxE = 4;

__device__ inline unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(unsigned)(v & 0xFFFFFFFFull), m, kWave);
  const int hi = __shfl_xor((int)(unsigned)(v >> 32), m, kWave);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// Ascending bitonic sort of E*NT keys (NT threads), element (e, tid) at
// index e*NT+tid.
template <int NT>
__device__ inline void block_bitonic(unsigned long long (&v)[kMaxE], int E,
                                     unsigned long long* lds) {
  const int tid = threadIdx.x;
  const int npad = E * NT;
  for (int kk = 2; kk <= npad; kk <<= 1) {
    int j = kk >> 1;
    // partner in another register of this thread
    for (; j >= NT; j >>= 1) {
      const int je = j / NT;
#pragma unroll
      for (int e = 0; e < kMaxE; e++) {
        const int pe = e ^ je;
        if (e < E && pe > e) {
          const int i = e * NT + tid;
          const bool up = (i & kk) == 0;
          const unsigned long long a = v[e], b = v[pe];
          if ((a > b) == up) {
            v[e] = b;
            v[pe] = a;
          }
        }
      }
    }
    // partner in another wave: through LDS
    if (j >= kWave) {
#pragma unroll
      for (int e = 0; e < kMaxE; e++)
        if (e < E) lds[e * NT + tid] = v[e];
      __syncthreads();
      for (; j >= kWave; j >>= 1) {
        for (int t = tid; t < (npad >> 1); t += NT) {
          const int i = 2 * j * (t / j) + (t % j);
          const int l = i + j;
          const unsigned long long a = lds[i], b = lds[l];
          if ((a > b) == ((i & kk) == 0)) {
            lds[i] = b;
            lds[l] = a;
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int e = 0; e < kMaxE; e++)
        if (e < E) v[e] = lds[e * NT + tid];
      __syncthreads();
    }
    // partner in the same wave: cross-lane exchange
    for (; j > 0; j >>= 1) {
#pragma unroll
      for (int e = 0; e < kMaxE; e++) {
        if (e < E) {
          const int i = e * NT + tid;
          const unsigned long long o = shfl_xor_u64(v[e], j);
          const bool lower = (i & j) == 0;
          const bool up = (i & kk) == 0;
          // lower element keeps min when ascending, max when descending
          const bool take_min = (lower == up);
          const unsigned long long mn = v[e] < o ? v[e] : o;
          const unsigned long long mx = v[e] < o ? o : v[e];
          v[e] = take_min ? mn : mx;
        }
      }
    }
  }
}

// Stable LSD radix sort of m ints inside ONE workgroup of NT threads, 8-bit
// digits of key(v) (bits [0, kbits)), ping-pong between `a` and `b` (global
// memory; a holds the input).  Each pass: a digit histogram (LDS atomics:
// order-free), its exclusive scan, then the elements in tiles of NT, in
// order: a wave ranks its 64 elements among the same digit with 8 ballots
// (the lanes that agree on every bit; rank = those below the lane), the
// per-wave digit counts are scanned over the waves in wave order, and each
// element goes to base[digit] + earlier waves + its rank -- equal keys keep
// their input order.  O(m) per pass.  Returns the array holding the result.
// lds: (2 + NT / 64) * 256 ints.
template <int NT, typename KeyF>
__device__ int* wg_radix_sort(int* a, int* b, int m, int kbits, KeyF key, int* lds) {
  constexpr int NW = NT / kWave;
  static_assert(NT >= 256 && NT % kWave == 0, "one thread per digit");
  int* base = lds;             // [256] running bucket offsets
  int* tot = lds + 256;        // [256] this tile's digit totals
  int* wtab = lds + 512;       // [NW][256] per-wave digit counts, then their prefixes
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int sh = 0; sh < kbits; sh += 8) {
    for (int i = tid; i < 256 + NW * 256; i += NT) (i < 256 ? base[i] : wtab[i - 256]) = 0;
    __syncthreads();
    for (int e = tid; e < m; e += NT) atomicAdd(&base[(key(a[e]) >> sh) & 255], 1);
    __syncthreads();
    {
      // exclusive scan of the 256 counts: wave scans, then the wave sums
      int c = tid < 256 ? base[tid] : 0;
      const int own = c;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const int t = __shfl_up(c, off, kWave);
        if (lane >= off) c += t;
      }
      if (tid < 256 && lane == 63) tot[wv] = c;
      __syncthreads();
      int add = 0;
      if (tid < 256)
        for (int w = 0; w < wv; w++) add += tot[w];
      __syncthreads();
      if (tid < 256) base[tid] = add + c - own;
      __syncthreads();
    }
    for (int t0 = 0; t0 < m; t0 += NT) {
      const int e = t0 + tid;
      const bool ok = e < m;
      const int v = ok ? a[e] : 0;
      const int dg = ok ? (key(v) >> sh) & 255 : 0;
      unsigned long long peers = __ballot(ok);
#pragma unroll
      for (int bit = 0; bit < 8; bit++) {
        const bool one = (dg >> bit) & 1;
        const unsigned long long bb = __ballot(ok && one);
        peers &= one ? bb : ~bb;
      }
      const int rank = __popcll(peers & lt);
      if (ok && rank == 0) wtab[wv * 256 + dg] = __popcll(peers);
      __syncthreads();
      if (tid < 256) {
        int run = 0;
        for (int w = 0; w < NW; w++) {
          const int c = wtab[w * 256 + tid];
          wtab[w * 256 + tid] = run;
          run += c;
        }
        tot[tid] = run;
      }
      __syncthreads();
      if (ok) b[base[dg] + wtab[wv * 256 + dg] + rank] = v;
      __syncthreads();
      if (tid < 256) {
        base[tid] += tot[tid];
        for (int w = 0; w < NW; w++) wtab[w * 256 + tid] = 0;
      }
      __syncthreads();
    }
    __threadfence_block();  // b's global writes are read by other threads next pass
    __syncthreads();
    int* t = a;
    a = b;
    b = t;
  }
  return a;
}

}  // namespace pcr
