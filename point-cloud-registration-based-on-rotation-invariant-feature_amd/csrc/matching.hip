// matching.hip -- feature-space mutual nearest neighbours of registration
// pairs, for gfx950 (the step after the extractor in the
// reference's registration evaluation, datasets/deepgmr_mn40.py:232-244
// find_correspondence_one_pair):
//   diff[i][j] = |f1_i|^2 + |f2_j|^2 - 2 f1_i . f2_j
//   corr12 = argmin_j diff, corr21 = argmin_i diff (first index on ties)
//   mutual: corr21[corr12[i]] == i  ->  (idx1, idx2) in ascending i.
// The [n1, n2] cross term is a dense contraction over the channels: fp32
// MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products, a k-ordered fmaf chain)
// on 128 x 128 tiles staged through LDS; the epilogue turns each tile into
// per-row and per-column (diff, index) minima with wave shuffles and merges
// them across tiles with 64-bit atomicMin on ascending keys, so the
// [n1, n2] matrix never reaches HBM.  Numerics are restated bit for bit by
// the oracle (include/pcr_math.h: pcr_match_*).
#include "common.hpp"

namespace pcr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMT = 128;  // tile rows (f1) and columns (f2)
// channels per LDS stage: 16 (two double-buffered stages of A and B take
// 34 KB, four workgroups per CU) measured 0.417 -> 0.350 ms at c4 (128 pairs
// x 1024 points, C = 64) and 1.59 -> 1.47 ms at C = 512 against 32 (68 KB,
// two per CU: the epilogue of one workgroup had too few MFMAs beside it)
constexpr int kKC = 16;
constexpr int kMPad = kMT + 4;
constexpr int kE = kKC * kMT / 256;  // channels of one row each thread stages per stage

// One stage of the operands: thread t holds kE consecutive channels of row
// t / 2 of A and of B (float4 loads when the stage is full and c % 4 == 0).
__device__ inline void match_load_stage(const float* __restrict__ A, const float* __restrict__ B,
                                        int i0, int j0, int n1, int n2, int c, int k0, int lr,
                                        int lk, float (&va)[kE], float (&vb)[kE]) {
  const int ka = k0 + lk;
  const bool ra = i0 + lr < n1, rb = j0 + lr < n2;
  if (ka + kE <= c && (c & 3) == 0) {
    const float4* pa = reinterpret_cast<const float4*>(A + (size_t)(i0 + lr) * c + ka);
    const float4* pb = reinterpret_cast<const float4*>(B + (size_t)(j0 + lr) * c + ka);
#pragma unroll
    for (int q = 0; q < kE / 4; q++) {
      const float4 x = ra ? pa[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 y = rb ? pb[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      va[4 * q] = x.x;
      va[4 * q + 1] = x.y;
      va[4 * q + 2] = x.z;
      va[4 * q + 3] = x.w;
      vb[4 * q] = y.x;
      vb[4 * q + 1] = y.y;
      vb[4 * q + 2] = y.z;
      vb[4 * q + 3] = y.w;
    }
  } else {
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const int k = ka + e;
      va[e] = (ra && k < c) ? A[(size_t)(i0 + lr) * c + k] : 0.0f;
      vb[e] = (rb && k < c) ? B[(size_t)(j0 + lr) * c + k] : 0.0f;
    }
  }
}

// Channel-major operands ([c][rows] per pair): thread t holds row t % 128
// of A and of B, channels kE (t / 128) .. + kE - 1 of the stage, so each
// channel row is read as 128 consecutive floats.
__device__ inline void match_load_stage_cm(const float* __restrict__ A,
                                           const float* __restrict__ B, int i0, int j0, int n1,
                                           int n2, int c, int k0, int lr, int lk, float (&va)[kE],
                                           float (&vb)[kE]) {
  const int ka = k0 + lk;
  const bool ra = i0 + lr < n1, rb = j0 + lr < n2;
#pragma unroll
  for (int e = 0; e < kE; e++) {
    const int k = ka + e;
    va[e] = (ra && k < c) ? A[(size_t)k * n1 + i0 + lr] : 0.0f;
    vb[e] = (rb && k < c) ? B[(size_t)k * n2 + j0 + lr] : 0.0f;
  }
}

// pcr_match_key's high word without branches: the float bits of d + 0 (-0 ->
// +0) mapped to an ascending unsigned order, NaN -> 0 (first)
__device__ inline unsigned match_key_hi(float d) {
  const unsigned u = __float_as_uint(d + 0.0f);
  const unsigned k = u ^ ((unsigned)((int)u >> 31) | 0x80000000u);
  return d != d ? 0u : k;
}

// The tile epilogue: per element the diff (pcr_match_diff) and its key's
// high word (elements outside the matrices: ~0), then
//  - the row minimum over this lane's two columns by one 32-bit compare (the
//    columns are ascending, so a tie keeps the first), as a 64-bit key, then
//    the transpose-reduction over the 32 lanes of a half (as below);
//  - the column minimum over this lane's 32 rows, visited in ascending row
//    order, by a strict 32-bit compare (the first row wins a tie);
// the same (diff, index) minima as pcr_match_key's 64-bit ordering, with no
// branches and no global loads (the norms are in LDS).  It replaced a
// per-element 64-bit key loop with bounds branches and the norms loaded from
// global memory inside it (c4 match call 0.346 -> see DESIGN.md 4.8).
__device__ inline void match_epilogue(const f32x16 (&acc)[2][2], const float (&sq_s)[2][kMT],
                                      int i0, int j0, int wi, int wj, int lane, int n1, int n2,
                                      unsigned long long* __restrict__ rb,
                                      unsigned long long* __restrict__ cb) {
  float sc[2];
#pragma unroll
  for (int tj = 0; tj < 2; tj++) sc[tj] = sq_s[1][wj * 64 + tj * 32 + (lane & 31)];
  unsigned cu[2] = {~0u, ~0u};
  int crow[2] = {0, 0};
  // one 32-row half (ti) at a time: 16 keys per lane, a transpose-reduction
  // over lane bits 0-3 (15 shuffles: each step swaps half of the remaining
  // rows with the partner), then lanes l and l ^ 16 (the other 16 columns)
  // combine; 32 registers of keys instead of 64
#pragma unroll
  for (int ti = 0; ti < 2; ti++) {
    unsigned long long R[16];
#pragma unroll
    for (int v = 0; v < 16; v++) {
      const int rl = wi * 64 + ti * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
      const float sr = sq_s[0][rl];
      const int c0 = j0 + wj * 64 + (lane & 31);
      const bool rok = i0 + rl < n1;
      unsigned u[2];
#pragma unroll
      for (int tj = 0; tj < 2; tj++) {
        // an element outside the matrices keys as ~0: above every real key
        // (+inf maps to 0xFF800000), so it never wins
        const bool ok = rok && c0 + 32 * tj < n2;
        u[tj] = ok ? match_key_hi(pcr_match_diff(sr, sc[tj], acc[ti][tj][v])) : ~0u;
        const bool lt = u[tj] < cu[tj];
        cu[tj] = lt ? u[tj] : cu[tj];
        crow[tj] = lt ? i0 + rl : crow[tj];
      }
      const bool second = u[1] < u[0];
      const unsigned um = second ? u[1] : u[0];
      R[v] = um == ~0u ? ~0ull
                       : ((unsigned long long)um << 32) | (unsigned)(second ? c0 + 32 : c0);
    }
#pragma unroll
    for (int h = 8; h >= 1; h >>= 1) {
      const bool up = (lane & h) != 0;
#pragma unroll
      for (int i = 0; i < h; i++) {
        const unsigned long long send = up ? R[i] : R[i + h];
        const unsigned long long keep = up ? R[i + h] : R[i];
        const unsigned long long recv = shfl_xor_u64(send, h);
        R[i] = recv < keep ? recv : keep;
      }
    }
    const unsigned long long o = shfl_xor_u64(R[0], 16);
    const unsigned long long rmin = o < R[0] ? o : R[0];
    const int v = lane & 15;
    const int row = i0 + wi * 64 + ti * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
    if ((lane & 16) == 0 && row < n1) atomicMin(rb + row, rmin);
  }
#pragma unroll
  for (int tj = 0; tj < 2; tj++) {
    const unsigned long long m0 =
        cu[tj] == ~0u ? ~0ull : ((unsigned long long)cu[tj] << 32) | (unsigned)crow[tj];
    const unsigned long long o = shfl_xor_u64(m0, 32);
    const unsigned long long m = o < m0 ? o : m0;
    const int col = j0 + wj * 64 + tj * 32 + lane;
    if (lane < 32 && col < n2) atomicMin(cb + col, m);
  }
}

// Channels run through LDS in stages of kKC, double-buffered: the next
// stage's global loads are in flight while the MFMAs consume this one, and
// one barrier per stage suffices (a buffer is rewritten two stages later,
// after every wave passed the barrier in between).  Three waves per SIMD:
// the accumulators stay in the unified VGPR file (143 VGPRs, no AGPRs)
// (DESIGN.md 4.8).
template <bool CM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void match_tile_kernel(
    const float* __restrict__ f1, const float* __restrict__ f2, int n1, int n2, int c,
    unsigned long long* __restrict__ rowbest, unsigned long long* __restrict__ colbest) {
  __shared__ float a_s[2][kKC][kMPad];  // [buf][k][i]
  __shared__ float b_s[2][kKC][kMPad];  // [buf][k][j]
  __shared__ float sq_s[2][kMT];        // the tile's row / column norms
  const int p = blockIdx.z;
  const int i0 = blockIdx.y * kMT, j0 = blockIdx.x * kMT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv >> 1, wj = wv & 1;  // 2 x 2 waves, 64 x 64 each
  // the norms the epilogue reads: thread t runs pcr_match_sqnorm's ordered
  // fmaf chain for row t of A (t < kMT) or row t - kMT of B over the channels
  // as each stage lands in LDS (zero padding adds exact zeros), so no norm
  // launches and no norm loads (pairs step: two launches fewer)
  float nrm = 0.0f;
  const float* const nrow = tid < kMT ? &a_s[0][0][tid] : &b_s[0][0][tid - kMT];
  const float* A = f1 + (size_t)p * n1 * c;
  const float* B = f2 + (size_t)p * n2 * c;
  f32x16 acc[2][2];
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int tj = 0; tj < 2; tj++)
#pragma unroll
      for (int v = 0; v < 16; v++) acc[ti][tj][v] = 0.0f;
  const int lr = CM ? (tid & (kMT - 1)) : (tid >> 1);
  const int lk = CM ? (tid / kMT) * kE : (tid & 1) * kE;
  float va[kE], vb[kE];
  auto load = [&](int k0) {
    if (CM)
      match_load_stage_cm(A, B, i0, j0, n1, n2, c, k0, lr, lk, va, vb);
    else
      match_load_stage(A, B, i0, j0, n1, n2, c, k0, lr, lk, va, vb);
  };
  load(0);
  int buf = 0;
  for (int k0 = 0; k0 < c; k0 += kKC, buf ^= 1) {
#pragma unroll
    for (int e = 0; e < kE; e++) {
      a_s[buf][lk + e][lr] = va[e];
      b_s[buf][lk + e][lr] = vb[e];
    }
    lds_barrier();
    if (k0 + kKC < c) load(k0 + kKC);
    // k ascending: every product enters its accumulator in channel order
#pragma unroll
    for (int kk = 0; kk < kKC; kk += 2) {
      const int kr = kk + (lane >> 5);
      float a[2], bq[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        a[t] = a_s[buf][kr][wi * 64 + t * 32 + (lane & 31)];
        bq[t] = b_s[buf][kr][wj * 64 + t * 32 + (lane & 31)];
      }
#pragma unroll
      for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ti], bq[tj], acc[ti][tj], 0, 0, 0);
    }
    const float* col = nrow + buf * kKC * kMPad;  // a_s / b_s [buf][0][row]
#pragma unroll
    for (int e = 0; e < kKC; e++) {
      const float v = col[e * kMPad];
      nrm = __builtin_fmaf(v, v, nrm);
    }
  }
  {
    const float r = __builtin_sqrtf(nrm);  // pcr_match_sqnorm: sqrt of the sum, squared
    sq_s[tid < kMT ? 0 : 1][tid & (kMT - 1)] = r * r;
  }
  lds_barrier();
  // epilogue: C/D layout col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 (lane >> 5)
  match_epilogue(acc, sq_s, i0, j0, wi, wj, lane, n1, n2, rowbest + (size_t)p * n1,
                 colbest + (size_t)p * n2);
}

// corr12 / corr21 from the minima; mutual pairs compacted in ascending i
// (one workgroup per pair)
__global__ __launch_bounds__(1024) void match_finalize_kernel(
    const unsigned long long* __restrict__ rowbest, const unsigned long long* __restrict__ colbest,
    int n1, int n2, int* __restrict__ corr12, int* __restrict__ corr21, int* __restrict__ idx1,
    int* __restrict__ idx2, int* __restrict__ count) {
  __shared__ int scan_s[1024 / kWave + 1];
  const int p = blockIdx.x, tid = threadIdx.x;
  const unsigned long long* rb = rowbest + (size_t)p * n1;
  const unsigned long long* cb = colbest + (size_t)p * n2;
  int* c12 = corr12 + (size_t)p * n1;
  int* c21 = corr21 + (size_t)p * n2;
  for (int j = tid; j < n2; j += 1024) c21[j] = (int)(unsigned)(cb[j] & 0xFFFFFFFFull);
  int base = 0;
  for (int i0 = 0; i0 < n1; i0 += 1024) {
    const int i = i0 + tid;
    int m = 0, ci = 0;
    if (i < n1) {
      ci = (int)(unsigned)(rb[i] & 0xFFFFFFFFull);
      c12[i] = ci;
      m = (ci >= 0 && ci < n2 && (int)(unsigned)(cb[ci] & 0xFFFFFFFFull) == i) ? 1 : 0;
    }
    const int incl = block_inclusive_scan(m, scan_s);
    if (m) {
      idx1[(size_t)p * n1 + base + incl - 1] = i;
      idx2[(size_t)p * n1 + base + incl - 1] = ci;
    }
    __shared__ int tot_s;
    if (tid == 1023) tot_s = incl;
    __syncthreads();
    base += tot_s;
    __syncthreads();
  }
  for (int i = base + tid; i < n1; i += 1024) idx1[(size_t)p * n1 + i] = idx2[(size_t)p * n1 + i] = -1;
  if (tid == 0) count[p] = base;
}

static size_t match_ws_layout(int p, int n1, int n2, unsigned long long** rb,
                              unsigned long long** cb, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off = (off + bytes + 255) / 256 * 256;
    return q;
  };
  unsigned long long* r = (unsigned long long*)take((size_t)p * n1 * 8);
  unsigned long long* c = (unsigned long long*)take((size_t)p * n2 * 8);
  if (rb) {
    *rb = r;
    *cb = c;
  }
  return off;
}

}  // namespace pcr

using namespace pcr;

extern "C" size_t pcr_mutual_nn_workspace_size(int p, int n1, int n2) {
  if (p <= 0 || n1 <= 0 || n2 <= 0) return 256;
  return match_ws_layout(p, n1, n2, nullptr, nullptr, nullptr);
}

static pcr_status mutual_nn(bool cm, const float* f1, const float* f2, int p, int n1, int n2,
                            int c, int* corr12, int* corr21, int* idx1, int* idx2, int* count,
                            void* workspace, size_t workspace_bytes, void* stream,
                            const char* name) {
  PCR_REQUIRE(p >= 0 && n1 >= 1 && n2 >= 1 && c >= 1, "%s: invalid sizes", name);
  PCR_REQUIRE(p <= 65535, "%s: too many pairs (%d)", name, p);
  if (p == 0) return PCR_OK;
  unsigned long long *rb, *cb;
  const size_t need = match_ws_layout(p, n1, n2, &rb, &cb, (char*)workspace);
  PCR_REQUIRE(workspace != nullptr && workspace_bytes >= need,
              "%s: workspace too small (%zu < %zu)", name, workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  // the row and column minima are adjacent in the workspace: one fill
  if (hipMemsetAsync(rb, 0xFF, (size_t)((char*)(cb + (size_t)p * n2) - (char*)rb), st) !=
      hipSuccess)
    return launch_status(name);
  const dim3 grid(ceil_div(n2, kMT), ceil_div(n1, kMT), p);
  if (cm)
    hipLaunchKernelGGL(match_tile_kernel<true>, grid, dim3(256), 0, st, f1, f2, n1, n2, c, rb, cb);
  else
    hipLaunchKernelGGL(match_tile_kernel<false>, grid, dim3(256), 0, st, f1, f2, n1, n2, c, rb, cb);
  hipLaunchKernelGGL(match_finalize_kernel, dim3(p), dim3(1024), 0, st, rb, cb, n1, n2, corr12,
                     corr21, idx1, idx2, count);
  return launch_status(name);
}

extern "C" pcr_status pcr_mutual_nn_match(const float* f1, const float* f2, int p, int n1, int n2,
                                          int c, int* corr12, int* corr21, int* idx1, int* idx2,
                                          int* count, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  return mutual_nn(false, f1, f2, p, n1, n2, c, corr12, corr21, idx1, idx2, count, workspace,
                   workspace_bytes, stream, "mutual_nn_match");
}

extern "C" pcr_status pcr_mutual_nn_match_cm(const float* f1, const float* f2, int p, int n1,
                                             int n2, int c, int* corr12, int* corr21, int* idx1,
                                             int* idx2, int* count, void* workspace,
                                             size_t workspace_bytes, void* stream) {
  return mutual_nn(true, f1, f2, p, n1, n2, c, corr12, corr21, idx1, idx2, count, workspace,
                   workspace_bytes, stream, "mutual_nn_match_cm");
}
