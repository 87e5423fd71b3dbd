// devoxelize.hip -- spherical / cube trilinear devoxelization (forward and
// backward) and the PVConv dgcnn centre gather, for gfx950.
//
// Replaces (relative to the reference's PVCNN/modules/functional/src):
//   interpolate/spherical_trilinear_devox.cu:23-136, :150-194
//   interpolate/trilinear_devox.cu:22-106, :120-163
// and the torch gather block of PVCNN/modules/pvconv.py:68-89.
//
// Forward: one thread per point, channel groups across workgroups so the
// grid has >> 256 workgroups.  Corner indices/weights come from the shared
// bit-exact helpers (pcr_sph_corners / pcr_cube_corners).  The spherical
// quirk (integer-division gama_lo, radian fractions) confines every corner to
// cells [0, r^2 + 8r + 5): those gathers are L2 hits.
//
// Backward: the reference memsets a dense [B, C, r^3] grad and scatters 8*C
// float atomics per point onto <= 80 hot cells -- the worst contention case of
// global atomics.  Here one workgroup owns a (cloud, channel-group) slab: it
// accumulates the hot window [0, hw) in LDS, streams zeros over the rest of
// its slab with 16-byte stores, then (after its own stores are complete)
// adds the rare out-of-window corners with global atomics and finally stores
// the window.  The dense gradient is written exactly once.  Cube grads up
// to r = 32 with a workspace are a gather instead (devox_cube_order_kernel /
// devox_cube_gather_kernel): no float atomics at all.
#include "common.hpp"

namespace pcr {

template <bool SPH>
__global__ __launch_bounds__(256) void devox_fwd_kernel(const float* __restrict__ coords,
                                                        const float* __restrict__ feat,
                                                        const int* __restrict__ g_inds, int c,
                                                        int n, int r, int cg,
                                                        float* __restrict__ outs,
                                                        int* __restrict__ inds,
                                                        float* __restrict__ wgts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j0 = blockIdx.y * cg;
  const int b = blockIdx.z;
  if (i >= n) return;
  const int r3 = r * r * r;
  const float* x = coords + (size_t)b * 3 * n;
  int idx[8];
  float w[8];
  bool write_out = true;  // false -> outs stay 0 (reference: `continue`)
  bool ok;
  if (SPH) {
    const int pos = g_inds[(size_t)b * n + i];
    if (pos == -1) {
      ok = false;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        idx[q] = q == 0 ? -1 : 0;
        w[q] = 0.0f;
      }
    } else {
      ok = pcr_sph_corners(x[i], x[i + n], x[i + 2 * n], pos, r, idx, w) != 0;
      if (!ok) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
          idx[q] = 0;
          w[q] = 0.0f;
        }
      }
    }
    write_out = ok;
  } else {
    pcr_cube_corners(x[i], x[i + n], x[i + 2 * n], r, idx, w);
    ok = true;
  }
  if (blockIdx.y == 0) {
    int* I = inds + (size_t)b * 8 * n;
    float* Wt = wgts + (size_t)b * 8 * n;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      I[i + (size_t)q * n] = idx[q];
      Wt[i + (size_t)q * n] = w[q];
    }
  }
  bool inb[8];
#pragma unroll
  for (int q = 0; q < 8; q++) inb[q] = idx[q] >= 0 && idx[q] < r3;
  const int j1 = min(c, j0 + cg);
  for (int j = j0; j < j1; j++) {
    const float* f = feat + ((size_t)b * c + j) * r3;
    float v = 0.0f;
    if (write_out) {
      float fv[8];
#pragma unroll
      for (int q = 0; q < 8; q++) fv[q] = inb[q] ? f[idx[q]] : 0.0f;
      v = pcr_wsum8(w, fv);
    }
    outs[((size_t)b * c + j) * n + i] = v;
  }
}

// Spherical forward with the corner voxels in LDS.  Every corner of a
// valid point lies in a fixed set of 80 voxels (spherical_trilinear_devox.cu:
// 67-105: gama_lo = (pos / r^2) / r is integer division, so 0; the alpha
// index (int)(2 pi ga / r) + {0, 1} is 0..7; the beta index (int)(pi gb / r)
// + {0, 1} is 0..4; gama adds 0 or r^2): voxel g r^2 + a r + b, slot
// g * 40 + a * 5 + b.  One workgroup per (block of kSphFwdPts * 256 points,
// group of up to kSphFwdCG channels, cloud) stages those 80 values of its
// channels in LDS (a few KB from L2, shared by the cloud's workgroups), then
// every point computes its corners once and every channel's eight gathers
// are LDS reads; the outputs are coalesced stores.  A corner outside the set
// (g_inds >= r^3, an invalid input) is read from global memory, bounds-
// checked as devox_fwd_kernel does.  Same corners, weights and wsum8 order,
// so the same bits as devox_fwd_kernel<true>.  (That kernel gathered every
// corner from global memory: 8 C scattered 4-byte loads per point, bound by
// the L1 / TA request rate, 0.31 ms at c5.)
constexpr int kSphFwdThreads = 256;
constexpr int kSphFwdPts = 4;   // points per thread
constexpr int kSphFwdCG = 64;   // channels per workgroup: 80 x 64 x 4 = 20 KB of LDS
constexpr int kSphSlots = 80;
__device__ inline int sph_slot(int v, int r) {
  const int r2 = r * r;
  const int g = v / r2;
  const int rem = v - g * r2;
  const int a = rem / r;
  const int bb = rem - a * r;
  return (v >= 0 && g <= 1 && a <= 7 && bb <= 4) ? g * 40 + a * 5 + bb : -1;
}
__global__ __launch_bounds__(kSphFwdThreads) void devox_fwd_sph_lds_kernel(
    const float* __restrict__ coords, const float* __restrict__ feat,
    const int* __restrict__ g_inds, int c, int n, int r, float* __restrict__ outs,
    int* __restrict__ inds, float* __restrict__ wgts) {
  __shared__ float val_s[kSphFwdCG * kSphSlots];  // [channel][slot]
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * kSphFwdCG;
  const int cn = min(kSphFwdCG, c - c0);
  const int tid = threadIdx.x;
  const int r2 = r * r, r3 = r2 * r;
  const float* F = feat + ((size_t)b * c + c0) * r3;
  for (int t = tid; t < cn * kSphSlots; t += kSphFwdThreads) {
    const int ch = t / kSphSlots;
    const int sl = t - ch * kSphSlots;
    const int g = sl / 40, a = (sl - g * 40) / 5, bb = sl - g * 40 - a * 5;
    const int v = g * r2 + a * r + bb;
    val_s[t] = v < r3 ? F[(size_t)ch * r3 + v] : 0.0f;
  }
  __syncthreads();
  const float* x = coords + (size_t)b * 3 * n;
  float* O = outs + ((size_t)b * c + c0) * n;
#pragma unroll 1
  for (int pp = 0; pp < kSphFwdPts; pp++) {
    const int i = (blockIdx.x * kSphFwdPts + pp) * kSphFwdThreads + tid;
    if (i >= n) break;
    int idx[8];
    float w[8];
    bool ok;
    const int pos = g_inds[(size_t)b * n + i];
    if (pos == -1) {
      ok = false;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        idx[q] = q == 0 ? -1 : 0;
        w[q] = 0.0f;
      }
    } else {
      ok = pcr_sph_corners(x[i], x[i + n], x[i + 2 * n], pos, r, idx, w) != 0;
      if (!ok) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
          idx[q] = 0;
          w[q] = 0.0f;
        }
      }
    }
    if (blockIdx.y == 0) {
      int* I = inds + (size_t)b * 8 * n;
      float* Wt = wgts + (size_t)b * 8 * n;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        I[i + (size_t)q * n] = idx[q];
        Wt[i + (size_t)q * n] = w[q];
      }
    }
    int sl[8];
    bool all_lds = true;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      sl[q] = sph_slot(idx[q], r);
      all_lds &= sl[q] >= 0;
    }
    if (__all(all_lds || !ok)) {
      // every live point of the wave reads LDS only
      for (int ch = 0; ch < cn; ch++) {
        const float* vs = val_s + ch * kSphSlots;
        float fv[8];
#pragma unroll
        for (int q = 0; q < 8; q++) fv[q] = vs[ok ? sl[q] : 0];
        O[(size_t)ch * n + i] = ok ? pcr_wsum8(w, fv) : 0.0f;
      }
    } else {
      for (int ch = 0; ch < cn; ch++) {
        const float* vs = val_s + ch * kSphSlots;
        float fv[8];
#pragma unroll
        for (int q = 0; q < 8; q++)
          fv[q] = sl[q] >= 0 ? vs[sl[q]]
                             : ((idx[q] >= 0 && idx[q] < r3) ? F[(size_t)ch * r3 + idx[q]] : 0.0f);
        O[(size_t)ch * n + i] = ok ? pcr_wsum8(w, fv) : 0.0f;
      }
    }
  }
}

// The extractor's devoxelisation from the dense grid it just wrote: the
// same 80-slot LDS staging as devox_fwd_sph_lds_kernel, with the corner
// indices / weights prep already computed (dinds / dwgts) and the per-cloud
// max-pooled descriptor.  One workgroup of 1024 threads per (cloud, group of
// up to 64 channels) covers every point of its cloud (n <= 4096), so the
// descriptor needs no cross-workgroup step.  Lane = channel: the points are
// taken in chunks of 1024 whose corner slots and weights go to LDS once;
// then each wave walks 64 consecutive points of the chunk, reading a point's
// slots and weights as broadcasts and its eight corner values at
// channel * 81 + slot, which are 32 distinct banks for 32 consecutive
// channels (81 = 17 mod 32, odd): no conflicts.  (Lane = point made the
// eight reads random slots of one channel row, ~4-way conflicts: 211 us at
// the c3 shape.)  Four consecutive points' outputs of a channel leave as one
// 16-byte store.  Replaces re-forming every voxel mean from the features per
// channel group (vox_grid_kernel<2>, 0.94 ms at the c3 shape) with a read of
// the 80 corner values per channel.  Same corners, weights and wsum8 order
// as the reference path, so the same bits; the descriptor is a max (order
// free).
constexpr int kGridDevoxThreads = 1024;
constexpr int kGridDevoxChunk = 1024;  // points whose corners sit in LDS at once
constexpr int kGridDevoxOut = 255;     // slot byte of a corner outside the 80-slot set
constexpr int kGridDevoxMaxN = 4096;
__global__ __launch_bounds__(kGridDevoxThreads) void devox_grid_desc_kernel(
    const float* __restrict__ grid, const int* __restrict__ dinds,
    const float* __restrict__ dwgts, int c, int n, int r, float* __restrict__ devox,
    float* __restrict__ desc) {
  // [channel][81]: the 80 corner slots and a zero (the slot of every
  // zero-weight corner, e.g. all of a dropped point's: +0 * 0 terms, so the
  // point's output is +0 like the reference's untouched zero)
  constexpr int kStride = kSphSlots + 1;
  constexpr int kW = kGridDevoxThreads / kWave;
  __shared__ float val_s[kSphFwdCG * kStride];
  __shared__ __align__(16) float pw_s[kGridDevoxChunk][8];              // corner weights
  __shared__ __align__(8) unsigned char psl_s[kGridDevoxChunk][8];     // corner slots
  __shared__ int pgi_s[kGridDevoxChunk][8];                            // corner voxels (slow path)
  __shared__ float red_s[kW][kSphFwdCG];
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * kSphFwdCG;
  const int cn = min(kSphFwdCG, c - c0);
  const int tid = threadIdx.x;
  const int wv = tid >> 6, lane = tid & 63;
  const int r2 = r * r, r3 = r2 * r;
  const float* F = grid + ((size_t)b * c + c0) * r3;
  for (int t = tid; t < cn * kStride; t += kGridDevoxThreads) {
    const int ch = t / kStride;
    const int sl = t - ch * kStride;
    const int g = sl / 40, a = (sl - g * 40) / 5, bb = sl - g * 40 - a * 5;
    const int v = g * r2 + a * r + bb;
    val_s[t] = (sl < kSphSlots && v < r3) ? F[(size_t)ch * r3 + v] : 0.0f;
  }
  const int* I = dinds + (size_t)b * 8 * n;
  const float* Wt = dwgts + (size_t)b * 8 * n;
  const int ch = lane;
  const bool live = ch < cn;
  const float* vs = val_s + (live ? ch : 0) * kStride;
  const float* Fc = F + (size_t)(live ? ch : 0) * r3;
  float* O = devox + ((size_t)b * c + c0 + (live ? ch : 0)) * n;
  // 16-byte stores when every channel row starts 16-byte aligned
  const bool vec4 = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(devox) & 15) == 0;
  float m = -__builtin_inff();
  for (int p0 = 0; p0 < n; p0 += kGridDevoxChunk) {
    // corners of the chunk's points (prep's dinds / dwgts; a dropped point
    // has inds {-1, 0, ...} and zero weights)
    bool all_lds = true;
    {
      const int i = p0 + tid;
      if (tid < kGridDevoxChunk && i < n) {
        unsigned lo = 0u, hi = 0u;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int v = I[i + (size_t)q * n];
          const float w = Wt[i + (size_t)q * n];
          int sl = w == 0.0f ? kSphSlots : sph_slot(v, r);
          if (sl < 0) {
            all_lds = false;
            sl = kGridDevoxOut;
          }
          pw_s[tid][q] = w;
          pgi_s[tid][q] = v;
          if (q < 4)
            lo |= (unsigned)sl << (8 * q);
          else
            hi |= (unsigned)sl << (8 * (q - 4));
        }
        *(uint2*)psl_s[tid] = uint2{lo, hi};
      }
    }
    const bool fast = __syncthreads_and(all_lds);  // also the staging barrier
    const int pn = min(kGridDevoxChunk, n - p0);
    // wave wv: points [wv * 64, wv * 64 + 64) of the chunk, four at a time
    const int q0 = wv * kWave;
    for (int qq = q0; qq < min(pn, q0 + kWave); qq += 4) {
      float v4[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int pi = qq + u;
        v4[u] = 0.0f;
        if (pi < pn) {
          const uint2 sp = *(const uint2*)psl_s[pi];
          const float4 wa = *(const float4*)&pw_s[pi][0];
          const float4 wb = *(const float4*)&pw_s[pi][4];
          const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
          float fv[8];
#pragma unroll
          for (int q = 0; q < 8; q++) {
            const int sl = (int)(((q < 4 ? sp.x : sp.y) >> (8 * (q & 3))) & 0xFFu);
            if (fast || sl != kGridDevoxOut) {
              fv[q] = vs[sl];
            } else {
              const int gi = pgi_s[pi][q];
              fv[q] = (gi >= 0 && gi < r3) ? Fc[gi] : 0.0f;
            }
          }
          v4[u] = pcr_wsum8(w, fv);
          m = fmaxf(m, v4[u]);
        }
      }
      if (live) {
        const int i = p0 + qq;
        if (vec4 && qq + 4 <= pn) {
          *(float4*)(O + i) = float4{v4[0], v4[1], v4[2], v4[3]};
        } else {
#pragma unroll
          for (int u = 0; u < 4; u++)
            if (qq + u < pn) O[i + u] = v4[u];
        }
      }
    }
    lds_only_barrier();  // the chunk's corner reads are done before the next chunk's writes
  }
  if (desc) {
    red_s[wv][ch] = m;
    lds_only_barrier();
    if (tid < cn) {
      float mm = red_s[0][tid];
      for (int q = 1; q < kW; q++) mm = fmaxf(mm, red_s[q][tid]);
      desc[(size_t)b * c + c0 + tid] = mm;
    }
  }
}

// Cube forward for grids whose channel row fits in LDS (r <= 32): one
// workgroup per (cloud, channel) stages the whole row with coalesced 16-byte
// loads, so the 8 corner gathers of every point are LDS reads instead of
// scattered 4-byte global gathers (a cloud's 8 point blocks used to fetch
// each row's lines again).  Corners are recomputed per channel (a few VALU);
// channel 0 writes inds / wgts.  Same corners and wsum8 order as
// devox_fwd_kernel<false>, so the same bits.
constexpr int kFwdRowThreads = 1024;
__global__ __launch_bounds__(kFwdRowThreads) void devox_fwd_cube_row_kernel(
    const float* __restrict__ coords, const float* __restrict__ feat, int c, int n, int r,
    float* __restrict__ outs, int* __restrict__ inds, float* __restrict__ wgts) {
  extern __shared__ __align__(16) float row_s[];  // [r^3]
  const int j = blockIdx.x;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int r3 = r * r * r;
  const float* f = feat + ((size_t)b * c + j) * r3;
  // 16-byte loads only when every row starts 16-byte aligned (the C ABI
  // accepts any 4-byte-aligned features pointer)
  if ((r3 & 3) == 0 && (reinterpret_cast<uintptr_t>(feat) & 15) == 0) {
    const float4* f4 = (const float4*)f;
    float4* s4 = (float4*)row_s;
    for (int t = tid; t < (r3 >> 2); t += kFwdRowThreads) s4[t] = f4[t];
  } else {
    for (int t = tid; t < r3; t += kFwdRowThreads) row_s[t] = f[t];
  }
  __syncthreads();
  const float* x = coords + (size_t)b * 3 * n;
  float* o = outs + ((size_t)b * c + j) * n;
  for (int i = tid; i < n; i += kFwdRowThreads) {
    int idx[8];
    float w[8];
    pcr_cube_corners(x[i], x[i + n], x[i + 2 * n], r, idx, w);
    if (j == 0) {
      int* I = inds + (size_t)b * 8 * n;
      float* Wt = wgts + (size_t)b * 8 * n;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        I[i + (size_t)q * n] = idx[q];
        Wt[i + (size_t)q * n] = w[q];
      }
    }
    float fv[8];
#pragma unroll
    for (int q = 0; q < 8; q++) fv[q] = (idx[q] >= 0 && idx[q] < r3) ? row_s[idx[q]] : 0.0f;
    o[i] = pcr_wsum8(w, fv);
  }
}

// Backward with the dense grad written once (see header comment).
constexpr int kBwdThreads = 256;
constexpr int kBwdMaxG = 4;

__global__ __launch_bounds__(kBwdThreads) void devox_bwd_kernel(
    const float* __restrict__ grad_y, const int* __restrict__ inds, const float* __restrict__ wgts,
    int c, int n, int r, int G, int hw, int skip_neg, float* __restrict__ grad_x,
    const int* __restrict__ order) {
  extern __shared__ __align__(16) float acc_s[];  // [G][hw]
  // spherical grads: each wave's segment sums for the 80 corner voxels
  // (every regular spherical corner lies there; devox_fwd_sph_lds_kernel),
  // folded into the window in wave order at the end.  One wave's LDS
  // atomics complete in issue order and the lanes of one instruction in a
  // fixed order, so the sums -- and the gradient -- are the same on every
  // run; tail adds of all waves into the one window raced.
  __shared__ float priv_s[kBwdThreads / kWave][kBwdMaxG][kSphSlots];
  const int r3 = r * r * r;
  const bool use_priv = skip_neg && r >= 8;  // slot -> voxel is one-to-one
  const int grp = blockIdx.x;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int c0 = grp * G;
  const int gcount = min(G, c - c0);
  for (int t = tid; t < G * hw; t += kBwdThreads) acc_s[t] = 0.0f;
  for (int t = tid; t < (kBwdThreads / kWave) * kBwdMaxG * kSphSlots; t += kBwdThreads)
    (&priv_s[0][0][0])[t] = 0.0f;
  __syncthreads();
  const int* I = inds + (size_t)b * 8 * n;
  const float* Wt = wgts + (size_t)b * 8 * n;
  const float* gy = grad_y + ((size_t)b * c + c0) * n;
  float* gx = grad_x + ((size_t)b * c + c0) * r3;
  // 1. accumulate the hot window in LDS; note whether any corner falls outside
  int outside = 0;
  if (skip_neg) {
    // Spherical grads: the 64 points of a wave mostly share a handful of
    // corner sets (the integer-division quirk pins gamma_lo = 0, so every
    // corner set is one of ~28 (alpha_lo, beta_lo) cells plus three "hi"
    // flags).  One LDS float atomic per (point, corner, channel) serialises
    // on those shared addresses, at about 0.44 lane-ops per CU-cycle.  So the
    // wave sorts its points by corner set (bitonic over lanes), sums w * g
    // per segment with a segmented shuffle scan, and only the segment tails
    // add into the window: distinct addresses, no collisions.  Points whose
    // corners do not follow that pattern take the per-point atomics.
    const int lane = tid & 63, wv = tid >> 6;
    constexpr long long kNoKey = (1ll << 57) - 1;  // above every key (ci0 < 2^22)
    // `order` (devox_bwd_order_kernel): the cloud's points sorted by corner
    // set, so a wave's 64 consecutive entries are already sorted and the
    // per-wave sort is skipped (segments are also longer: fewer tails)
    // (I and Wt are then the sorted copies, indexed by position; only the
    // gradients are gathered by point)
    const int* ord = order ? order + (size_t)b * n : nullptr;
    for (int base = wv * kWave; base < n; base += kBwdThreads) {
      const int i = base + lane;
      const int pt = ord ? (i < n ? ord[i] : 0) : i;
      const bool live = i < n && I[i] != -1;
      int ci[8];
      float cw[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        ci[q] = live ? I[i + (size_t)q * n] : 0;
        cw[q] = live ? Wt[i + (size_t)q * n] : 0.0f;
      }
      const int d1 = ci[1] - ci[0], d2 = ci[2] - ci[0], d4 = ci[4] - ci[0];
      // regular corner set: idx1 = idx0 + b, idx2 = idx0 + a, idx4 = idx0 + g,
      // idx3 = idx2 + b, idx5 = idx4 + b, idx6 = idx4 + a, idx7 = idx6 + b
      const bool reg = live && (d1 == 0 || d1 == 1) && d2 >= 0 && d4 >= 0 && ci[3] == ci[2] + d1 &&
            ci[5] == ci[4] + d1 && ci[6] == ci[4] + d2 && ci[7] == ci[6] + d1 && ci[0] >= 0 &&
            ci[7] < hw && hw < (1 << 22) && d2 < 4096 && d4 < (1 << 22);
      float gv[kBwdMaxG];
#pragma unroll
      for (int g = 0; g < kBwdMaxG; g++) gv[g] = (live && g < gcount) ? gy[(size_t)g * n + pt] : 0.0f;
      if (live && !reg) {  // irregular: per-point atomics (as below)
#pragma unroll
        for (int q = 0; q < 8; q++) {
          outside |= (ci[q] >= hw && ci[q] < r3);
          if (ci[q] >= 0 && ci[q] < hw)
            for (int g = 0; g < gcount; g++) atomicAdd(&acc_s[g * hw + ci[q]], cw[q] * gv[g]);
        }
      }
      // sort key: corner set (idx0, then the three deltas); ties by lane
      const long long key0 =
          reg ? (((long long)ci[0] << 35) | ((long long)d4 << 13) | ((long long)d2 << 1) | d1)
              : kNoKey;
      long long k2 = (key0 << 6) | lane;
      if (!ord)
#pragma unroll
      for (int k = 2; k <= kWave; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
          const long long o = (long long)shfl_xor_u64((unsigned long long)k2, j);
          const bool lower = (lane & j) == 0, asc = (lane & k) == 0;
          const long long mn = o < k2 ? o : k2, mx = o < k2 ? k2 : o;
          k2 = (lower == asc) ? mn : mx;
        }
      }
      const int src = (int)(k2 & 63);
      const long long mykey = k2 >> 6;
      const bool mine = mykey < kNoKey;
      float v[8][kBwdMaxG];
      {
        float w8[8], g4[kBwdMaxG];
#pragma unroll
        for (int q = 0; q < 8; q++) w8[q] = __shfl(cw[q], src, kWave);
#pragma unroll
        for (int g = 0; g < kBwdMaxG; g++) g4[g] = __shfl(gv[g], src, kWave);
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
          for (int g = 0; g < kBwdMaxG; g++) v[q][g] = mine ? w8[q] * g4[g] : 0.0f;
      }
      const int c0 = __shfl(ci[0], src, kWave);
      const long long prevk = (long long)__shfl_up((unsigned long long)mykey, 1, kWave);
      const long long nextk = (long long)__shfl_down((unsigned long long)mykey, 1, kWave);
      int seg = (lane == 0 || prevk != mykey) ? lane : 0;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const int o = __shfl_up(seg, d, kWave);
        if (lane >= d) seg = max(seg, o);
      }
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const bool add = lane - d >= seg;
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
          for (int g = 0; g < kBwdMaxG; g++) {
            const float o = __shfl_up(v[q][g], d, kWave);
            if (add) v[q][g] += o;
          }
      }
      const bool tail = mine && (lane == kWave - 1 || nextk != mykey);
      if (tail) {
        const int e1 = (int)(mykey & 1), e2 = (int)((mykey >> 1) & 0xFFF),
                  e4 = (int)((mykey >> 13) & 0x3FFFFF);
        const int cq[8] = {c0, c0 + e1, c0 + e2, c0 + e2 + e1,
                           c0 + e4, c0 + e4 + e1, c0 + e4 + e2, c0 + e4 + e2 + e1};
        int sq[8];
        bool in80 = use_priv;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          sq[q] = sph_slot(cq[q], r);
          in80 &= sq[q] >= 0;
        }
        if (in80) {
#pragma unroll
          for (int q = 0; q < 8; q++)
#pragma unroll
            for (int g = 0; g < kBwdMaxG; g++)
              if (g < gcount) atomicAdd(&priv_s[wv][g][sq[q]], v[q][g]);
        } else {
#pragma unroll
          for (int q = 0; q < 8; q++)
#pragma unroll
            for (int g = 0; g < kBwdMaxG; g++)
              if (g < gcount) atomicAdd(&acc_s[g * hw + cq[q]], v[q][g]);
        }
      }
    }
    if (use_priv) {
      __syncthreads();
      for (int t = tid; t < gcount * kSphSlots; t += kBwdThreads) {
        const int g = t / kSphSlots, sl = t - g * kSphSlots;
        float sum = priv_s[0][g][sl];
#pragma unroll
        for (int w = 1; w < kBwdThreads / kWave; w++) sum += priv_s[w][g][sl];
        const int gg = sl / 40, a = (sl - gg * 40) / 5, bb = sl - gg * 40 - a * 5;
        const int vx = gg * r * r + a * r + bb;
        if (vx < hw) acc_s[g * hw + vx] += sum;
      }
    }
  }
  if (!skip_neg)
  for (int i = tid; i < n; i += kBwdThreads) {
    if (skip_neg && I[i] == -1) continue;
    int ci[8];
    float cw[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      ci[q] = I[i + (size_t)q * n];
      cw[q] = Wt[i + (size_t)q * n];
      outside |= (ci[q] >= hw && ci[q] < r3);
    }
    for (int g = 0; g < gcount; g++) {
      const float gv = gy[(size_t)g * n + i];
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (ci[q] >= 0 && ci[q] < hw) atomicAdd(&acc_s[g * hw + ci[q]], cw[q] * gv);
    }
  }
  const int any_outside = __syncthreads_or(outside);
  // 2. zero-stream the slab outside the window (written exactly once)
  for (int g = 0; g < gcount; g++) {
    float* row = gx + (size_t)g * r3;
    int start = hw;
    while (start < r3 && (start & 3)) {
      if (tid == 0) row[start] = 0.0f;
      start++;
    }
    const int nv = (r3 - start) >> 2;
    // nontemporal zero stream: the dense gradient grid is written once and
    // not read back here (c3 step 1.97 -> 1.90 ms with the PPF / emit ones)
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v* w4 = (f4v*)(row + start);
    const f4v z4 = {0.f, 0.f, 0.f, 0.f};
    for (int t = tid; t < nv; t += kBwdThreads) __builtin_nontemporal_store(z4, &w4[t]);
    for (int t = start + nv * 4 + tid; t < r3; t += kBwdThreads) row[t] = 0.0f;
  }
  // 3. rare out-of-window corners (cube grids): global atomics after this
  //    workgroup's own zero stores are released to the device
  if (any_outside) {
    __threadfence();
    __syncthreads();
    for (int i = tid; i < n; i += kBwdThreads) {
      if (skip_neg && I[i] == -1) continue;
      for (int q = 0; q < 8; q++) {
        const int v = I[i + (size_t)q * n];
        if (v < hw || v >= r3) continue;
        const float w = Wt[i + (size_t)q * n];
        const int pt = order ? order[(size_t)b * n + i] : i;  // I / Wt by position, gy by point
        for (int g = 0; g < gcount; g++) atomicAdd(gx + (size_t)g * r3 + v, w * gy[(size_t)g * n + pt]);
      }
    }
  }
  __syncthreads();
  // 3. store the window
  for (int g = 0; g < gcount; g++)
    for (int t = tid; t < hw; t += kBwdThreads)
      __builtin_nontemporal_store(acc_s[g * hw + t], &gx[(size_t)g * r3 + t]);
}

__global__ __launch_bounds__(256) void center_gather_kernel(const float* __restrict__ features,
                                                            const float* __restrict__ grid,
                                                            const int* __restrict__ ind, int c,
                                                            int n, int r3, int cg,
                                                            float* __restrict__ related) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j0 = blockIdx.y * cg;
  const int b = blockIdx.z;
  if (i >= n) return;
  const int pos = ind[(size_t)b * n + i];
  const bool ok = pos >= 0 && pos < r3;
  const int j1 = min(c, j0 + cg);
  for (int j = j0; j < j1; j++) {
    const size_t o = ((size_t)b * c + j) * n + i;
    related[o] = ok ? features[o] - grid[((size_t)b * c + j) * r3 + pos] : 0.0f;
  }
}

}  // namespace pcr

using namespace pcr;

static pcr_status devox_forward(bool sph, int r, const float* coords, const float* features,
                                const int* g_inds, int b, int c, int n, float* outs, int* inds,
                                float* wgts, void* stream, const char* name) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r >= 1, "%s: invalid sizes", name);
  PCR_REQUIRE((int64_t)r * r * r < (1ll << 31) / 64, "%s: resolution too large", name);
  if (b == 0 || n == 0) return PCR_OK;
  const size_t row_bytes = (size_t)r * r * r * 4;
  if (!sph && c > 0 && row_bytes <= 128 * 1024) {
    allow_big_lds(devox_fwd_cube_row_kernel, row_bytes);
    hipLaunchKernelGGL(devox_fwd_cube_row_kernel, dim3(c, b), dim3(kFwdRowThreads), row_bytes,
                       as_stream(stream), coords, features, c, n, r, outs, inds, wgts);
    return launch_status(name);
  }
  if (sph) {
    dim3 grid(ceil_div(n, kSphFwdPts * kSphFwdThreads), c > 0 ? ceil_div(c, kSphFwdCG) : 1, b);
    hipLaunchKernelGGL(devox_fwd_sph_lds_kernel, grid, dim3(kSphFwdThreads), 0,
                       as_stream(stream), coords, features, g_inds, c, n, r, outs, inds, wgts);
    return launch_status(name);
  }
  const int cg = 8;
  dim3 grid(ceil_div(n, 256), c > 0 ? ceil_div(c, cg) : 1, b);
  if (sph)
    hipLaunchKernelGGL(devox_fwd_kernel<true>, grid, dim3(256), 0, as_stream(stream), coords,
                       features, g_inds, c, n, r, cg, outs, inds, wgts);
  else
    hipLaunchKernelGGL(devox_fwd_kernel<false>, grid, dim3(256), 0, as_stream(stream), coords,
                       features, g_inds, c, n, r, cg, outs, inds, wgts);
  return launch_status(name);
}

extern "C" pcr_status pcr_spherical_trilinear_devoxelize_forward(int r, int is_training,
                                                                 const float* coords,
                                                                 const float* features,
                                                                 const int* g_inds, int b, int c,
                                                                 int n, float* outs, int* inds,
                                                                 float* wgts, void* stream) {
  (void)is_training;
  return devox_forward(true, r, coords, features, g_inds, b, c, n, outs, inds, wgts, stream,
                       "spherical_trilinear_devoxelize_forward");
}

extern "C" pcr_status pcr_extractor_grid_devox(const float* grid, const int* dinds,
                                               const float* dwgts, int b, int c, int n, int r,
                                               float* devox, float* desc, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 1 && n >= 1 && n <= kGridDevoxMaxN && r >= 1,
              "extractor_grid_devox: invalid sizes b=%d c=%d n=%d r=%d (n <= %d)", b, c, n, r,
              kGridDevoxMaxN);
  PCR_REQUIRE((int64_t)r * r * r < (1ll << 31) / 64, "extractor_grid_devox: resolution too large");
  if (b == 0) return PCR_OK;
  hipLaunchKernelGGL(devox_grid_desc_kernel, dim3(ceil_div(c, kSphFwdCG), b),
                     dim3(kGridDevoxThreads), 0, as_stream(stream), grid, dinds, dwgts, c, n, r,
                     devox, desc);
  return launch_status("extractor_grid_devox");
}

extern "C" pcr_status pcr_trilinear_devoxelize_forward(int r, int is_training, const float* coords,
                                                       const float* features, int b, int c, int n,
                                                       float* outs, int* inds, float* wgts,
                                                       void* stream) {
  (void)is_training;
  return devox_forward(false, r, coords, features, nullptr, b, c, n, outs, inds, wgts, stream,
                       "trilinear_devoxelize_forward");
}

// The points of each cloud sorted by spherical corner set (the key the
// backward's wave sort uses, compressed to 52 bits: cell 20, gamma step 20,
// alpha step 11, beta step 1) with the point id below it; irregular and
// dropped points last.  One workgroup per cloud.
constexpr int kOrderMaxN = kSortBlock * kMaxE;
__global__ __launch_bounds__(kSortBlock) void devox_bwd_order_kernel(const int* __restrict__ inds,
                                                                     const float* __restrict__ wgts,
                                                                     int n, int npad,
                                                                     int* __restrict__ order,
                                                                     int* __restrict__ sinds,
                                                                     float* __restrict__ swgts) {
  extern __shared__ __align__(16) unsigned long long okeys[];  // [npad]
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int E = npad / kSortBlock;
  const int* I = inds + (size_t)b * 8 * n;
  unsigned long long kv[kMaxE];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int i = e * kSortBlock + tid;
    kv[e] = ~0ull;
    if (e < E && i < n) {
      int ci[8];
#pragma unroll
      for (int q = 0; q < 8; q++) ci[q] = I[i + (size_t)q * n];
      const int d1 = ci[1] - ci[0], d2 = ci[2] - ci[0], d4 = ci[4] - ci[0];
      const bool reg = ci[0] != -1 && (d1 == 0 || d1 == 1) && d2 >= 0 && d4 >= 0 &&
                       ci[3] == ci[2] + d1 && ci[5] == ci[4] + d1 && ci[6] == ci[4] + d2 &&
                       ci[7] == ci[6] + d1 && ci[0] >= 0 && ci[0] < (1 << 20) &&
                       d2 < (1 << 11) && d4 < (1 << 20);
      const unsigned long long key =
          reg ? (((unsigned long long)ci[0] << 32) | ((unsigned long long)d4 << 12) |
                 ((unsigned long long)d2 << 1) | (unsigned long long)d1)
              : (1ull << 52) - 1;
      kv[e] = (key << 12) | (unsigned long long)i;
    }
  }
  block_bitonic<kSortBlock>(kv, E, okeys);
  // the point order, and the corner data in that order (the backward then
  // reads it coalesced; only the gradients are gathered)
  int* o = order + (size_t)b * n;
  int* si = sinds + (size_t)b * 8 * n;
  float* sw = swgts + (size_t)b * 8 * n;
  const float* W = wgts + (size_t)b * 8 * n;
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int pos = e * kSortBlock + tid;
    if (e < E && pos < n) {
      const int p = (int)(kv[e] & 0xFFFull);
      o[pos] = p;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        si[pos + (size_t)q * n] = I[p + (size_t)q * n];
        sw[pos + (size_t)q * n] = W[p + (size_t)q * n];
      }
    }
  }
}

// Cube grads as a gather (trilinear_devox.cu:120-163 scatters w * g into
// grad_x with one float atomic per (point, corner, channel)).  The 8n
// (point, corner) pairs of a cloud are counting-sorted by voxel once, here,
// one workgroup per cloud with the r^3 counters in LDS; the gather kernel
// then gives every voxel one thread that sums its segment for a group of
// channels and writes grad_x exactly once, coalesced, with no atomics.
// seg [b][r3 + 1]: first pair of each voxel (seg[r3] = pairs kept);
// pairs [b][8n]: (point id, weight bits) in voxel order.  Pairs whose
// voxel is outside [0, r3) are dropped, as the window kernel drops them.
constexpr int kCubeOrderThreads = 1024;
// counters padded by one word per 32 so the scan's per-thread runs of 32
// contiguous voxels start in distinct banks
__device__ inline int cube_pad(int v) { return v + (v >> 5); }
__global__ __launch_bounds__(kCubeOrderThreads) void devox_cube_order_kernel(
    const int* __restrict__ inds, const float* __restrict__ wgts, int n, int r3,
    int* __restrict__ seg, int2* __restrict__ pairs) {
  extern __shared__ __align__(16) int cnt_s[];  // [cube_pad(r3)] counters | [17] scan
  int* scan_s = cnt_s + cube_pad(r3);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int m = 8 * n;
  const int* I = inds + (size_t)b * m;
  const float* W = wgts + (size_t)b * m;
  for (int v = tid; v < cube_pad(r3); v += kCubeOrderThreads) cnt_s[v] = 0;
  lds_barrier();
  for (int p = tid; p < m; p += kCubeOrderThreads) {
    const int v = I[p];
    if (v >= 0 && v < r3) atomicAdd(&cnt_s[cube_pad(v)], 1);
  }
  lds_barrier();
  // exclusive scan: thread t owns the contiguous voxels [t * per, t * per + per)
  const int per = (r3 + kCubeOrderThreads - 1) / kCubeOrderThreads;
  const int v0 = min(tid * per, r3), v1 = min(v0 + per, r3);
  int local = 0;
  for (int v = v0; v < v1; v++) local += cnt_s[cube_pad(v)];
  const int incl = block_inclusive_scan(local, scan_s);
  int run = incl - local;
  for (int v = v0; v < v1; v++) {
    const int k = cnt_s[cube_pad(v)];
    cnt_s[cube_pad(v)] = run;
    run += k;
  }
  int* S = seg + (size_t)b * (r3 + 1);
  if (tid == kCubeOrderThreads - 1) S[r3] = incl;
  lds_barrier();
  for (int v = tid; v < r3; v += kCubeOrderThreads) S[v] = cnt_s[cube_pad(v)];
  lds_barrier();
  // placement by wave 0 alone, pairs in ascending order: one wave's LDS
  // atomics complete in issue order, and the lanes of one instruction that
  // hit the same counter are served in the LDS unit's fixed order, so every
  // voxel's pairs land in the same order on every run -- the same summation
  // order, hence the same bits.  (Placement atomics from 16 waves raced for a voxel's slots, and
  // the gather's sum order changed from run to run.)  Eight pairs per lane
  // per round: their loads are issued together and their atomics back to
  // back, so the round trip is paid once per 512 pairs.
  if (tid >= kWave) return;
  int2* P = pairs + (size_t)b * m;
  constexpr int U = 8;
  for (int p0 = 0; p0 < m; p0 += U * kWave) {
    int v[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int p = p0 + u * kWave + tid;
      v[u] = p < m ? I[p] : -1;
      w[u] = p < m ? W[p] : 0.0f;
    }
    int pos[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      pos[u] = (v[u] >= 0 && v[u] < r3) ? atomicAdd(&cnt_s[cube_pad(v[u])], 1) : -1;
#pragma unroll
    for (int u = 0; u < U; u++)
      if (pos[u] >= 0) P[pos[u]] = make_int2((p0 + u * kWave + tid) % n, __float_as_int(w[u]));
  }
}

// One thread per voxel and G channels.  A voxel's pairs form a dependent
// chain (pair load -> gradient gathers), so the kernel is bound by chain
// latency times waves, not by bytes: G = 64 channels per thread quarters the
// waves of G = 16, and the next pair is loaded while the current pair's G
// gathers are in flight.
constexpr int kCubeGatherThreads = 256;
template <int G>
__global__ __launch_bounds__(kCubeGatherThreads) void devox_cube_gather_kernel(
    const float* __restrict__ grad_y, const int* __restrict__ seg, const int2* __restrict__ pairs,
    int c, int n, int r3, float* __restrict__ grad_x) {
  const int v = blockIdx.x * kCubeGatherThreads + threadIdx.x;
  const int c0 = blockIdx.y * G;
  const int b = blockIdx.z;
  if (v >= r3) return;
  const int gcount = min(G, c - c0);
  const int* S = seg + (size_t)b * (r3 + 1);
  const int s = S[v], e = S[v + 1];
  const int2* P = pairs + (size_t)b * 8 * n;
  const float* gy = grad_y + ((size_t)b * c + c0) * n;
  float acc[G];
#pragma unroll
  for (int g = 0; g < G; g++) acc[g] = 0.0f;
  int2 nxt = s < e ? P[s] : make_int2(0, 0);
  for (int j = s; j < e; j++) {
    const int2 pw = nxt;
    if (j + 1 < e) nxt = P[j + 1];
    const float w = __int_as_float(pw.y);
    float gv[G];
#pragma unroll
    for (int g = 0; g < G; g++) gv[g] = g < gcount ? gy[(size_t)g * n + pw.x] : 0.0f;
#pragma unroll
    for (int g = 0; g < G; g++) acc[g] += w * gv[g];
  }
  float* gx = grad_x + ((size_t)b * c + c0) * r3 + v;
#pragma unroll
  for (int g = 0; g < G; g++)
    if (g < gcount) gx[(size_t)g * r3] = acc[g];
}

// The same gather with everything it reads in LDS: one workgroup per
// (cloud, group of kCubeLdsG channels) keeps those gradient rows in LDS and
// walks the cloud's voxels in chunks of four consecutive voxels per thread
// (float4 grad_x stores).  A chunk's seg
// entries and its contiguous pair range (up to kCubePairCap pairs; a larger
// range is read from global memory) are loaded into registers one chunk
// ahead, and the chunk boundaries two chunks ahead, so the global loads of
// chunk i + 1 are in flight while chunk i sums from LDS and streams its
// grad_x rows out.  Same pair order, so the same bits as
// devox_cube_gather_kernel.
constexpr int kCubeLdsThreads = 1024;
constexpr int kCubeLdsG = 4;
constexpr int kCubeVpt = 4;  // voxels per thread: a chunk is 4096 voxels
constexpr int kCubeChunk = kCubeVpt * kCubeLdsThreads;
constexpr int kCubePairRegs = 4;
constexpr int kCubePairCap = kCubePairRegs * kCubeLdsThreads;
__global__ __launch_bounds__(kCubeLdsThreads) void devox_cube_gather_lds_kernel(
    const float* __restrict__ grad_y, const int* __restrict__ seg, const int2* __restrict__ pairs,
    int c, int n, int r3, float* __restrict__ grad_x) {
  // [G][n] | seg [chunk] (the chunk's end stays in a register) | pairs [cap]:
  // 80 KB at n = 2048, two workgroups per CU
  extern __shared__ __align__(16) float gy_s[];
  int* seg_s = (int*)(gy_s + kCubeLdsG * n);
  int2* pair_s = (int2*)(seg_s + kCubeChunk);
  constexpr int T = kCubeLdsThreads;
  constexpr int CH = kCubeChunk;
  const int c0 = blockIdx.x * kCubeLdsG;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int gcount = min(kCubeLdsG, c - c0);
  const float* gy = grad_y + ((size_t)b * c + c0) * n;
  const int* S = seg + (size_t)b * (r3 + 1);
  const int2* P = pairs + (size_t)b * 8 * n;
  float* gx = grad_x + ((size_t)b * c + c0) * r3;
  const bool vec = (r3 & 3) == 0;
  // chunk 0 in registers, chunk 1's boundaries
  int sreg[kCubeVpt];
#pragma unroll
  for (int k = 0; k < kCubeVpt; k++) sreg[k] = S[min(k * T + tid, r3)];
  int cur0 = S[0], cur1 = S[min(CH, r3)];
  int nxt0 = cur1, nxt1 = S[min(2 * CH, r3)];
  int2 preg[kCubePairRegs];
#pragma unroll
  for (int k = 0; k < kCubePairRegs; k++) {
    const int t = k * T + tid;
    preg[k] = (cur1 - cur0 <= kCubePairCap && t < cur1 - cur0) ? P[cur0 + t] : make_int2(0, 0);
  }
  for (int t = tid; t < kCubeLdsG * n; t += T) gy_s[t] = t < gcount * n ? gy[t] : 0.0f;
  for (int v0 = 0; v0 < r3; v0 += CH) {
    lds_only_barrier();  // the previous chunk's LDS reads are done
    const int p0 = cur0, np = cur1 - cur0;
    const bool staged = np <= kCubePairCap;
#pragma unroll
    for (int k = 0; k < kCubeVpt; k++) seg_s[k * T + tid] = sreg[k];
#pragma unroll
    for (int k = 0; k < kCubePairRegs; k++)
      if (staged && k * T + tid < np) pair_s[k * T + tid] = preg[k];
    const int vn = v0 + CH;
    if (vn < r3) {  // chunk i + 1 into registers, chunk i + 2's boundaries
#pragma unroll
      for (int k = 0; k < kCubeVpt; k++) sreg[k] = S[min(vn + k * T + tid, r3)];
      const int m = nxt1 - nxt0;
#pragma unroll
      for (int k = 0; k < kCubePairRegs; k++) {
        const int t = k * T + tid;
        if (m <= kCubePairCap && t < m) preg[k] = P[nxt0 + t];
      }
      cur0 = nxt0;
      cur1 = nxt1;
      nxt0 = nxt1;
      nxt1 = S[min(vn + 2 * CH, r3)];
    }
    lds_only_barrier();
    const int vb = v0 + kCubeVpt * tid;  // this thread's 4 consecutive voxels
    if (vb < r3) {
      float acc[kCubeVpt][kCubeLdsG];
#pragma unroll
      for (int q = 0; q < kCubeVpt; q++) {
#pragma unroll
        for (int g = 0; g < kCubeLdsG; g++) acc[q][g] = 0.0f;
        const int sq = kCubeVpt * tid + q;
        const int s = seg_s[sq], e = sq + 1 < CH ? seg_s[sq + 1] : p0 + np;
        // separate loops: a global pair load in the staged loop would make
        // every iteration wait for the whole vmcnt (the prefetch included)
        if (staged) {
          for (int j = s; j < e; j++) {
            const int2 pw = pair_s[j - p0];
            const float w = __int_as_float(pw.y);
#pragma unroll
            for (int g = 0; g < kCubeLdsG; g++) acc[q][g] += w * gy_s[g * n + pw.x];
          }
        } else {
          for (int j = s; j < e; j++) {
            const int2 pw = P[j];
            const float w = __int_as_float(pw.y);
#pragma unroll
            for (int g = 0; g < kCubeLdsG; g++) acc[q][g] += w * gy_s[g * n + pw.x];
          }
        }
      }
      if (vec) {
#pragma unroll
        for (int g = 0; g < kCubeLdsG; g++)
          if (g < gcount)
            *(float4*)(gx + (size_t)g * r3 + vb) =
                make_float4(acc[0][g], acc[1][g], acc[2][g], acc[3][g]);
      } else {
#pragma unroll
        for (int q = 0; q < kCubeVpt; q++)
#pragma unroll
          for (int g = 0; g < kCubeLdsG; g++)
            if (g < gcount && vb + q < r3) gx[(size_t)g * r3 + vb + q] = acc[q][g];
      }
    }
  }
}
static size_t cube_gather_lds_bytes(int n) {
  return (size_t)kCubeLdsG * n * 4 + kCubeChunk * 4 + (size_t)kCubePairCap * 8;
}

static pcr_status devox_backward(const float* grad_y, const int* inds, const float* wgts, int b,
                                 int c, int n, int r, int skip_neg, float* grad_x,
                                 const int* order, void* stream);

// order [b][n] | sorted inds [b][8][n] | sorted wgts [b][8][n]
extern "C" size_t pcr_devoxelize_backward_workspace_size(int b, int n) {
  if (b <= 0 || n <= 0) return 256;
  return ((size_t)b * n * 4 * 17 + 255) / 256 * 256;
}

// cube grids up to 32^3 additionally: seg [b][r3 + 1] | pairs [b][8n]
static size_t cube_seg_bytes(int b, int r3) { return ((size_t)b * (r3 + 1) * 4 + 255) / 256 * 256; }
static bool cube_gather_ok(int n, int r) {
  return r >= 1 && r <= 32 && n >= 1 && (int64_t)n * 8 < (1ll << 28);
}
extern "C" size_t pcr_devoxelize_backward_workspace_size_r(int b, int n, int r, int spherical) {
  const size_t base = pcr_devoxelize_backward_workspace_size(b, n);
  if (spherical || b <= 0 || !cube_gather_ok(n, r)) return base;
  const size_t cube = cube_seg_bytes(b, r * r * r) + (size_t)b * 8 * n * 8;
  return cube > base ? cube : base;
}

extern "C" pcr_status pcr_devoxelize_backward_ws(const float* grad_y, const int* inds,
                                                 const float* wgts, int b, int c, int n, int r,
                                                 int skip_neg, float* grad_x, void* workspace,
                                                 size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r >= 1, "devoxelize_backward: invalid sizes");
  const int* order = nullptr;
  // spherical grads of clouds the order kernel sorts in one workgroup (ids
  // in 12 bits); otherwise the per-wave sort
  if (skip_neg && n >= 1 && n <= kOrderMaxN && n <= 4096 && b > 0 && c > 0 && workspace &&
      workspace_bytes >= pcr_devoxelize_backward_workspace_size(b, n)) {
    int npad = kSortBlock;
    while (npad < n) npad <<= 1;
    int* ord = (int*)workspace;
    int* sinds = ord + (size_t)b * n;
    float* swgts = (float*)(sinds + (size_t)b * 8 * n);
    hipLaunchKernelGGL(devox_bwd_order_kernel, dim3(b), dim3(kSortBlock), (size_t)npad * 8,
                       as_stream(stream), inds, wgts, n, npad, ord, sinds, swgts);
    // the backward reads the sorted corner data by position
    return devox_backward(grad_y, sinds, swgts, b, c, n, r, skip_neg, grad_x, ord, stream);
  }
  if (!skip_neg && b > 0 && c > 0 && cube_gather_ok(n, r) && workspace &&
      workspace_bytes >= pcr_devoxelize_backward_workspace_size_r(b, n, r, 0)) {
    const int r3 = r * r * r;
    int* seg = (int*)workspace;
    int2* pairs = (int2*)((char*)workspace + cube_seg_bytes(b, r3));
    const size_t lds = ((size_t)r3 + (r3 >> 5) + kCubeOrderThreads / kWave + 1) * 4;
    allow_big_lds(devox_cube_order_kernel, lds);
    hipLaunchKernelGGL(devox_cube_order_kernel, dim3(b), dim3(kCubeOrderThreads), lds,
                       as_stream(stream), inds, wgts, n, r3, seg, pairs);
    const dim3 vb(ceil_div(r3, kCubeGatherThreads));
    const size_t lds_g = cube_gather_lds_bytes(n);
    if (lds_g <= 80 * 1024) {
      allow_big_lds(devox_cube_gather_lds_kernel, lds_g);
      hipLaunchKernelGGL(devox_cube_gather_lds_kernel, dim3(ceil_div(c, kCubeLdsG), b),
                         dim3(kCubeLdsThreads), lds_g, as_stream(stream), grad_y, seg, pairs, c,
                         n, r3, grad_x);
    } else if (c >= 48)
      hipLaunchKernelGGL(devox_cube_gather_kernel<64>, dim3(vb.x, ceil_div(c, 64), b),
                         dim3(kCubeGatherThreads), 0, as_stream(stream), grad_y, seg, pairs, c, n,
                         r3, grad_x);
    else
      hipLaunchKernelGGL(devox_cube_gather_kernel<16>, dim3(vb.x, ceil_div(c, 16), b),
                         dim3(kCubeGatherThreads), 0, as_stream(stream), grad_y, seg, pairs, c, n,
                         r3, grad_x);
    return launch_status("trilinear_devoxelize_backward");
  }
  return devox_backward(grad_y, inds, wgts, b, c, n, r, skip_neg, grad_x, order, stream);
}

extern "C" pcr_status pcr_devoxelize_backward(const float* grad_y, const int* inds,
                                              const float* wgts, int b, int c, int n, int r,
                                              int skip_neg, float* grad_x, void* stream) {
  return devox_backward(grad_y, inds, wgts, b, c, n, r, skip_neg, grad_x, nullptr, stream);
}

static pcr_status devox_backward(const float* grad_y, const int* inds, const float* wgts, int b,
                                 int c, int n, int r, int skip_neg, float* grad_x,
                                 const int* order, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r >= 1, "devoxelize_backward: invalid sizes");
  const int64_t r3l = (int64_t)r * r * r;
  PCR_REQUIRE(r3l < (1ll << 31) / 64, "devoxelize_backward: resolution too large");
  if (b == 0 || c == 0) return PCR_OK;
  const int r3 = (int)r3l;
  // hot window: every spherical corner lies below r^2 + 8r + 5.  Rounded up
  // to 32 voxels, so the zero stream past it starts on a 128-byte line: from
  // r^2 + 8r + 8 (1288 at r = 32) every 1 KB wave store split a line with the
  // next one, and the c3 backward took 0.617 ms alone against 0.528 aligned
  // (c3 step 1.91 -> 1.81-1.85 ms, profiles/r06_ab_devox_bwd_align.log)
  int hw = skip_neg ? (r * r + 8 * r + 8 + 31) / 32 * 32 : 2048;
  if (hw > r3) hw = r3;
  int G = kBwdMaxG;
  if (!skip_neg && hw < r3 && (size_t)r3 * 4 <= 128 * 1024) {
    // cube grids up to 32^3: cube corners land anywhere, so a 2048-voxel
    // window sent nearly every corner to global atomics (10 ms at c3).  One
    // channel's whole grid fits in LDS (128 KB, one workgroup per CU).
    hw = r3;
    G = 1;
  }
  while (G > 1 && (size_t)G * hw * 4 > 80 * 1024) G >>= 1;
  if ((size_t)G * hw * 4 > 128 * 1024) hw = 80 * 1024 / 4;
  if (hw > r3) hw = r3;
  allow_big_lds(devox_bwd_kernel, (size_t)G * hw * 4);
  hipLaunchKernelGGL(devox_bwd_kernel, dim3(ceil_div(c, G), b), dim3(kBwdThreads),
                     (size_t)G * hw * 4, as_stream(stream), grad_y, inds, wgts, c, n, r, G, hw,
                     skip_neg, grad_x, order);
  return launch_status("devoxelize_backward");
}

extern "C" pcr_status pcr_dgcnn_center_gather(const float* features, const float* avg_grid,
                                              const int* ind, int b, int c, int n, int r3,
                                              float* related, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r3 >= 1, "dgcnn_center_gather: invalid sizes");
  if (b == 0 || c == 0 || n == 0) return PCR_OK;
  const int cg = 8;
  hipLaunchKernelGGL(center_gather_kernel, dim3(ceil_div(n, 256), ceil_div(c, cg), b), dim3(256),
                     0, as_stream(stream), features, avg_grid, ind, c, n, r3, cg, related);
  return launch_status("dgcnn_center_gather");
}
