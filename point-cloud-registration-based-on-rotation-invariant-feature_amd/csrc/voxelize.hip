// voxelize.hip -- spherical / cube average voxelization and the fused
// extractor voxel stage, for gfx950.
//
// Replaces (paths relative to the reference's PVCNN/modules/functional/src):
//   spherical_voxelization/spherical_vox.cu:19-125  grid stats + scatter-mean
//   voxelization/vox.cu:18-73                       cube grid stats + scatter-mean
//   spherical_vox.cu:139-163, vox.cu:87-111         backward gathers
// and the coordinate normalisation of PVCNN/modules/spherical_vox.py:16-20.
//
// Design (MI355X-first, not a translation):
//   The reference zero-fills a dense [B, C, r^3] grid and scatters C float
//   atomics per point (one 4-byte atomic per cache line).  Here the work is
//   split in two launches:
//   1. vox_prep_kernel -- one workgroup per cloud: voxel index per point
//      (bit-exact shared math, include/pcr_math.h), a stable LDS bitonic sort
//      of (voxel, point) keys, the occupied-voxel segment list and an
//      occupancy bitmap with per-word prefix counts (rank structure).
//   2. vox_grid_kernel -- one workgroup per (cell tile, channel group, cloud):
//      stages its channels' feature rows in LDS, forms each occupied voxel's
//      mean in ascending point order (bit-identical to the serial oracle),
//      then streams its [G, tile] slab of the grid exactly once with 16-byte
//      coalesced stores, zeros included.  No atomics, no memset, no re-read.
//      HBM traffic = the algorithmic bytes (grid + cnt written once, features
//      read once).  The extractor variant also evaluates the spherical
//      devoxelisation of the grid it just formed (from LDS, not HBM) and the
//      per-cloud max-pooled descriptor.
#include "common.hpp"


namespace pcr {

constexpr int kPrepThreads = kSortBlock;
constexpr int kSmallPrepThreads = 256;
constexpr int kSmallPrepN = kSmallPrepThreads * kMaxE;
constexpr int kMaxSortN = kSortBlock * kMaxE;
constexpr int kGridThreads = 256;
constexpr int kDevoxThreads = 1024;
constexpr int kMaxG = 8;

enum PrepMode { kSphCoords = 0, kSphNormalize = 1, kCube = 2 };

struct VoxWs {
  int* perm;         // [b][n] point ids sorted by (voxel, id); dropped last
  int* seg_off;      // [b][n+1] start of each occupied voxel in perm
  int* seg_vox;      // [b][n] voxel of each segment
  int* nseg;         // [b]
  unsigned* bitmap;  // [b][W] occupancy bits
  int* wprefix;      // [b][W] occupied voxels before word w
  unsigned short* wpre16;  // [b][W] the same as u16 (clouds of < 65536 points): the grid
                           // stream loads it instead of scanning the bitmap again
  int* dseg;         // [b][8][n] segment of each devox corner (-1: empty / none)
  unsigned* dseg16;  // [b][n][4]: the same as u16 pairs, empty -> n (n <= 65535): one
                     // 16-byte load per point for the grid stream's devox role
  float* means;      // [b][c][ms] voxel means per occupied segment (extractor only)
  unsigned short* segcnt;  // [b][ms] points per occupied segment (extractor only)
  int ms;            // row stride of means / segcnt: n + 1 rounded up to 4
  int W;             // words per cloud = ceil(r^3 / 32)
};

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static size_t vox_ws_layout(int b, int n, int r, VoxWs* ws, void* base, int cm = 0) {
  const int64_t r3 = (int64_t)r * r * r;
  const int W = (int)((r3 + 31) / 32);
  size_t off = 0;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off = align_up(off + bytes, 256);
    return q;
  };
  int* perm = (int*)take((size_t)b * n * 4);
  int* seg_off = (int*)take((size_t)b * (n + 1) * 4);
  int* seg_vox = (int*)take((size_t)b * n * 4);
  int* nseg = (int*)take((size_t)b * 4);
  unsigned* bitmap = (unsigned*)take((size_t)b * W * 4);
  int* wprefix = (int*)take((size_t)b * W * 4);
  unsigned short* wpre16 = (unsigned short*)take((size_t)b * W * 2);
  int* dseg = (int*)take((size_t)b * 8 * n * 4);
  unsigned* dseg16 = (unsigned*)take((size_t)b * n * 16);
  const int ms = (n + 1 + 3) / 4 * 4;
  // + 16 KB: vox_stream_kernel's LDS-DMA reads a whole item's pieces, past
  // the last row when c is odd
  float* means = cm > 0 ? (float*)take((size_t)b * cm * ms * 4 + 16384) : nullptr;
  // (+ 256 B: the grid stream's LDS-DMA reads whole 256-byte pieces)
  unsigned short* segcnt = cm > 0 ? (unsigned short*)take((size_t)b * ms * 2 + 256) : nullptr;
  if (ws) {
    ws->means = means;
    ws->segcnt = segcnt;
    ws->ms = ms;
    ws->dseg = dseg;
    ws->dseg16 = dseg16;
    ws->perm = perm;
    ws->seg_off = seg_off;
    ws->seg_vox = seg_vox;
    ws->nseg = nseg;
    ws->bitmap = bitmap;
    ws->wprefix = wprefix;
    ws->wpre16 = wpre16;
    ws->W = W;
  }
  return off;
}

static inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// ------------------------------------------------------------ prep kernel
// One workgroup of 1024 threads per cloud; thread t owns points t + e*1024.
// Everything after the initial coalesced loads stays in registers / LDS:
// fixed-order fp64 mean (cloud_mean), fp32 max norm, voxel index and
// devox corners, then a bitonic sort of the 64-bit (voxel, point) keys whose
// stages run in registers (partner in the same thread), with DPP/shuffles
// (partner in the same wave) or through LDS (other waves) -- 10 barriers for
// 1024 keys instead of 55.

// Fixed-order per-axis mean of a cloud in double, the order the oracle
// restates (orc_cloud_mean): "virtual thread" T of 1024 sums points T,
// T+1024, ... ascending; each virtual wave halves its 64 partials (l += l+s
// for s = 32..1); the 16 virtual-wave sums are halved the same way.  With
// NT = 1024 threads the virtual threads are the real ones; with NT = 256
// (clouds of <= 1024 points) thread t holds virtual threads t + e*256, e = 0..3
// (one point each), so its register e joins virtual wave 4e + (t >> 6).
// Returns the three means on every thread.
template <int NT>
__device__ inline void cloud_mean(const float (&px)[kMaxE], const float (&py)[kMaxE],
                                  const float (&pz)[kMaxE], int E, int n, double* red,
                                  float* mean_out) {
  static_assert(NT == 1024 || NT == 512 || NT == 256, "prep workgroup size");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int R = 1024 / NT;  // virtual waves per real wave
  double s[R][3];
#pragma unroll
  for (int q = 0; q < R; q++) s[q][0] = s[q][1] = s[q][2] = 0.0;
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int q = e % R;
    if (e < E && e * NT + tid < n) {
      s[q][0] += (double)px[e];
      s[q][1] += (double)py[e];
      s[q][2] += (double)pz[e];
    }
  }
#pragma unroll
  for (int q = 0; q < R; q++) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_down(s[q][a], off, kWave);
        if (lane < off) s[q][a] += o;
      }
      if (lane == 0) red[a * 16 + q * (NT / kWave) + w] = s[q][a];
    }
  }
  lds_barrier();
  if (tid < 3) {
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = red[tid * 16 + i];
#pragma unroll
    for (int off = 8; off > 0; off >>= 1)
#pragma unroll
      for (int i = 0; i < off; i++) v[i] += v[i + off];
    mean_out[tid] = (float)(v[0] / (double)n);
  }
  lds_barrier();
}

template <int MODE, int NT>
__global__ __launch_bounds__(NT) void vox_prep_kernel(
    const float* __restrict__ coords_f, const int* __restrict__ coords_i, int n, int r, int npad,
    float* __restrict__ norm_out, int* __restrict__ ind, VoxWs ws, int* __restrict__ dinds,
    float* __restrict__ dwgts, int prio) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  unsigned long long* keys = (unsigned long long*)smem_raw;  // [npad]
  unsigned* bm = (unsigned*)(keys + npad);                     // [W]
  __shared__ int scan_s[NT / kWave + 1];
  __shared__ double red[48];
  __shared__ float s_stat[4];
  __shared__ int s_flag;  // a crowded voxel: the bitonic path

  if (!PCR_PRIO(3) && prio) latency_kernel_priority();
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  constexpr int nt = NT;
  const int r3 = r * r * r;
  const int W = ws.W;
  const int E = npad / NT;
  PCR_STAMP(0);

  float px[kMaxE], py[kMaxE], pz[kMaxE];
  int ci[kMaxE][3];
  if (MODE == kCube) {
    const int* x = coords_i + (size_t)b * 3 * n;
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      const int i = e * nt + tid;
      const bool ok = e < E && i < n;
      ci[e][0] = ok ? x[i] : 0;
      ci[e][1] = ok ? x[i + n] : 0;
      ci[e][2] = ok ? x[i + 2 * n] : 0;
    }
  } else {
    const float* x = coords_f + (size_t)b * 3 * n;
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      const int i = e * nt + tid;
      const bool ok = e < E && i < n;
      px[e] = ok ? x[i] : 0.0f;
      py[e] = ok ? x[i + n] : 0.0f;
      pz[e] = ok ? x[i + 2 * n] : 0.0f;
    }
  }
  for (int w = tid; w < W; w += nt) bm[w] = 0u;
  if (tid == 0) s_flag = 0;

  if (MODE == kSphNormalize) {
    cloud_mean<NT>(px, py, pz, E, n, red, s_stat);
    PCR_STAMP(1);
    const float m0 = s_stat[0], m1 = s_stat[1], m2 = s_stat[2];
    float mx = 0.0f;
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      if (e < E && e * nt + tid < n) {
        px[e] -= m0;
        py[e] -= m1;
        pz[e] -= m2;
        mx = fmaxf(mx, __builtin_sqrtf(pcr_sumsq3f(px[e], py[e], pz[e])));
      }
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) scan_s[tid >> 6] = __float_as_int(mx);
    lds_barrier();
    if (tid == 0) {
      float m = 0.0f;
      for (int w = 0; w < nt / kWave; w++) m = fmaxf(m, __int_as_float(scan_s[w]));
      s_stat[3] = m + 1e-20f;
    }
    lds_barrier();
    const float den = s_stat[3];
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      px[e] = px[e] / den;
      py[e] = py[e] / den;
      pz[e] = pz[e] / den;
    }
  }

  PCR_STAMP(2);
  // voxel index, devox corners, sort keys
  unsigned long long kv[kMaxE];
  bool corner_ok[kMaxE];  // the reference interpolates this point (else outputs stay 0)
  int corner_cell[MODE == kSphNormalize ? kMaxE : 1][8];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    kv[e] = ~0ull;
    corner_ok[e] = false;
    const int i = e * nt + tid;
    if (e < E && i < n) {
      int v;
      bool valid;
      if (MODE == kCube) {
        v = ci[e][0] * r * r + ci[e][1] * r + ci[e][2];
        valid = (v >= 0 && v < r3);
      } else {
        if (MODE == kSphNormalize && norm_out) {
          float* o = norm_out + (size_t)b * 3 * n;
          o[i] = px[e];
          o[i + n] = py[e];
          o[i + 2 * n] = pz[e];
        }
        if (MODE == kSphNormalize && dinds) {
          // index and corners from one evaluation of the spherical
          // coordinates (bit-identical to pcr_sph_index + pcr_sph_corners)
          int cidx[8];
          float cw[8];
          int okc;
          v = pcr_sph_index_corners(px[e], py[e], pz[e], r, cidx, cw, &okc);
          valid = v >= 0;
          int* I = dinds + (size_t)b * 8 * n;
          float* Wt = dwgts + (size_t)b * 8 * n;
          const bool ok = valid && okc;
          corner_ok[e] = ok;
#pragma unroll
          for (int q = 0; q < 8; q++) corner_cell[MODE == kSphNormalize ? e : 0][q] = cidx[q];
#pragma unroll
          for (int q = 0; q < 8; q++) {
            I[i + (size_t)q * n] = ok ? cidx[q] : ((q == 0 && !valid) ? -1 : 0);
            Wt[i + (size_t)q * n] = ok ? cw[q] : 0.0f;
          }
        } else {
          v = pcr_sph_index(px[e], py[e], pz[e], r);
          valid = v >= 0;
        }
      }
      ind[(size_t)b * n + i] = v;
      kv[e] = ((unsigned long long)(valid ? (unsigned)v : 0xFFFFFFFFu) << 32) | (unsigned)i;
    }
  }

  PCR_STAMP(3);
  int* perm = ws.perm + (size_t)b * n;
  int* seg_off = ws.seg_off + (size_t)b * (n + 1);
  int* seg_vox = ws.seg_vox + (size_t)b * n;
  unsigned* gbm = ws.bitmap + (size_t)b * W;
  int* gpre = ws.wprefix + (size_t)b * W;
  int* pre_l = (int*)(bm + W);            // [W] word prefix
  int* cnt_l = pre_l + W;                 // [n] points per occupied voxel
  int* perm_l = cnt_l + n;                // [n] points grouped by voxel

  // 1. occupancy bitmap.  The bitmap was zeroed at the top; the normalising
  // mode's reductions put barriers in between, the others need one here, or
  // a slow wave's zeroing can erase a fast wave's bit (seen on cube grids:
  // a voxel lost its bit and its points joined the next segment)
  if (MODE != kSphNormalize) lds_barrier();
  for (int i = tid; i < n; i += nt) cnt_l[i] = 0;
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const unsigned v = (unsigned)(kv[e] >> 32);
    if (e < E && v != 0xFFFFFFFFu) atomicOr(&bm[v >> 5], 1u << (v & 31));
  }
  lds_barrier();
  // 2. per-word exclusive prefix of popcounts (rank of a voxel among the
  //    occupied ones == its segment id, segments in voxel order)
  {
    const int wchunk = (W + nt - 1) / nt;
    const int w0 = min(W, tid * wchunk), w1 = min(W, w0 + wchunk);
    int pc = 0;
    for (int w = w0; w < w1; w++) pc += __popc(bm[w]);
    const int pincl = block_inclusive_scan(pc, scan_s);
    int run = pincl - pc;
    for (int w = w0; w < w1; w++) {
      const unsigned word = bm[w];
      gbm[w] = word;
      gpre[w] = run;
      ws.wpre16[(size_t)b * W + w] = (unsigned short)run;
      pre_l[w] = run;
      run += __popc(word);
    }
    if (tid == nt - 1) s_stat[0] = __int_as_float(pincl);  // number of segments
  }
  lds_barrier();
  const int nseg = __float_as_int(s_stat[0]);
  // devox corners -> their voxel's segment (the grid kernel's devox part
  // gathers the voxel means by segment without a bitmap lookup); the corner
  // cells are still in this thread's registers
  if (MODE == kSphNormalize && dinds) {
    int* D = ws.dseg + (size_t)b * 8 * n;
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      const int i = e * nt + tid;
      if (e < E && i < n) {
        // dropped or not interpolated (spherical_trilinear_devox.cu:41-65
        // `continue`): every corner -1, so the output is +0 as untouched
        const bool skip = !corner_ok[e];
        unsigned pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int cell = corner_cell[MODE == kSphNormalize ? e : 0][q];
          int sg = -1;
          if (!skip && cell >= 0 && cell < r3) {
            const unsigned word = bm[cell >> 5], bit = 1u << (cell & 31);
            if (word & bit) sg = pre_l[cell >> 5] + __popc(word & (bit - 1u));
          }
          D[i + (size_t)q * n] = sg;
          pk[q >> 1] |= (unsigned)(sg >= 0 ? sg : n) << (16 * (q & 1));
        }
        if (n <= 65535)
          *(uint4*)(ws.dseg16 + ((size_t)b * n + i) * 4) = uint4{pk[0], pk[1], pk[2], pk[3]};
      }
    }
  }
  PCR_STAMP(4);
  // 3. counts per segment; arrival slot within the segment (unstable)
  int seg_of[kMaxE], slot_of[kMaxE];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const unsigned v = (unsigned)(kv[e] >> 32);
    seg_of[e] = -1;
    if (e < E && v != 0xFFFFFFFFu) {
      const unsigned bit = 1u << (v & 31);
      const int sg = pre_l[v >> 5] + __popc(bm[v >> 5] & (bit - 1u));
      seg_of[e] = sg;
      slot_of[e] = atomicAdd(&cnt_l[sg], 1);
      seg_vox[sg] = (int)v;
    }
  }
  lds_barrier();
  // 4. exclusive scan of the counts -> segment offsets; largest segment
  int big = 0;
  {
    const int chunk = (nseg + nt - 1) / nt;
    const int s0 = min(nseg, tid * chunk), s1 = min(nseg, s0 + chunk);
    int sum = 0;
    for (int q = s0; q < s1; q++) {
      sum += cnt_l[q];
      big = max(big, cnt_l[q]);
    }
    const int incl = block_inclusive_scan(sum, scan_s);
    int run = incl - sum;
    lds_barrier();
    for (int q = s0; q < s1; q++) {
      const int c = cnt_l[q];
      cnt_l[q] = run;  // now the segment start
      seg_off[q] = run;
      run += c;
    }
    if (tid == nt - 1) {
      ws.nseg[b] = nseg;
      seg_off[nseg] = incl;
      s_stat[1] = __int_as_float(incl);  // number of valid points
    }
  }
  PCR_STAMP(5);
  // 5. place the points in arrival order, then every point finds its rank
  //    among its voxel's points (ascending point order, the order the means
  //    are accumulated in) by one sweep of that voxel's slots -- independent
  //    LDS reads, no serial per-voxel pass.  A cloud with a crowded voxel
  //    takes the bitonic path.
  if (__any(big > 32)) s_flag = 1;
  lds_barrier();
  const int crowded = s_flag;
  if (!crowded) {
#pragma unroll
    for (int e = 0; e < kMaxE; e++)
      if (seg_of[e] >= 0) perm_l[cnt_l[seg_of[e]] + slot_of[e]] = (int)(unsigned)(kv[e] & 0xFFFFFFFFull);
    lds_barrier();
    const int nvalid = __float_as_int(s_stat[1]);
#pragma unroll
    for (int e = 0; e < kMaxE; e++) {
      const int sg = seg_of[e];
      if (sg >= 0) {
        const int id = (int)(unsigned)(kv[e] & 0xFFFFFFFFull);
        const int o0 = cnt_l[sg], o1 = (sg + 1 < nseg) ? cnt_l[sg + 1] : nvalid;
        int rank = 0;
        for (int x = o0; x < o1; x++) rank += perm_l[x] < id ? 1 : 0;
        perm[o0 + rank] = id;
      }
    }
  } else {
    // unique 64-bit keys (the low word is the point id): sorting them is a
    // stable sort by voxel
    block_bitonic<NT>(kv, E, keys);
#pragma unroll
    for (int e = 0; e < kMaxE; e++)
      if (e < E) keys[e * nt + tid] = kv[e];
    lds_barrier();
    for (int p = tid; p < n; p += nt) perm[p] = (int)(unsigned)(keys[p] & 0xFFFFFFFFull);
  }
  PCR_STAMP(6);
}

// ------------------------------------------------------------ grid kernel
// One workgroup per (cell tile, channel group, cloud).
// PART: 1 = stream the grid (+cnt), 2 = devoxelise + descriptor, 3 = both
// (a variant with the two as separate workgroups of one launch measured
// slower: 68 vs 60 us).
// NT threads: 256 for the streaming parts; the devox-only part runs 1024
// (one point per thread, so every corner load of a point is in flight at once).
template <int PART, int NT, int MG>
__global__ __launch_bounds__(NT) void vox_grid_kernel(
    const float* __restrict__ feat, int c, int n, int r3, int G, int tile_cells, VoxWs ws,
    float* __restrict__ out, int* __restrict__ cnt_out, const int* __restrict__ dinds,
    const float* __restrict__ dwgts, float* __restrict__ devox, float* __restrict__ desc,
    int ntiles, int ngrp, int nitems) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  // work items (tile, channel group, cloud), tile fastest; a launch of fewer
  // workgroups than items loops over them, so the kernel holds few CU slots
  // while it streams and other streams' kernels fit beside it
  for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
  if (item != (int)blockIdx.x) __syncthreads();  // LDS of the previous item
  const int tile = item % ntiles;
  const int role = PART;
  const int grp = (item / ntiles) % ngrp;
  const int b = item / (ntiles * ngrp);
  const int tid = threadIdx.x;
  const int W = ws.W;
  const int cell0 = tile * tile_cells;
  const int cell1 = min(r3, cell0 + tile_cells);
  const int wb = cell0 >> 5;
  const int we = (cell1 + 31) >> 5;
  const int nw = we - wb;
  const int c0 = grp * G;
  const int gcount = min(G, c - c0);

  PCR_STAMP(8);
  const unsigned* gbm = ws.bitmap + (size_t)b * W;
  const int* gpre = ws.wprefix + (size_t)b * W;
  const int nseg = ws.nseg[b];
  const int s_begin = gpre[wb];
  const int s_end = (we >= W) ? nseg : gpre[we];
  const int S = s_end - s_begin;

  // LDS carve: feat_s[G][n] | mean_s[G][ns] | scnt_s[ns] | bm_s[nw] | pre_s[nw];
  // ns = n + 1: slot n of every mean / count row holds 0, the value of an
  // empty cell or corner, so the gathers below need no masking
  const int ns = n + 1;
  float* feat_s = (float*)smem_raw;
  float* mean_s = feat_s + (size_t)G * n;
  int* scnt_s = (int*)(mean_s + (size_t)G * ns);
  unsigned* bm_s = (unsigned*)(scnt_s + ns);
  int* pre_s = (int*)(bm_s + nw);

  for (int w = tid; w < nw; w += NT) {
    bm_s[w] = gbm[wb + w];
    pre_s[w] = gpre[wb + w] - s_begin;
  }
  const float* fb = feat + ((size_t)b * c + c0) * n;
  if ((n & 3) == 0) {
    const int n4 = n >> 2;
    for (int g = 0; g < gcount; g++) {
      const float4* src = (const float4*)(fb + (size_t)g * n);
      float4* dst = (float4*)(feat_s + (size_t)g * n);
      for (int i = tid; i < n4; i += NT) dst[i] = src[i];
    }
  } else {
    for (int g = 0; g < gcount; g++)
      for (int i = tid; i < n; i += NT) feat_s[(size_t)g * n + i] = fb[(size_t)g * n + i];
  }
  __syncthreads();

  PCR_STAMP(9);
  // voxel means, ascending point order inside each voxel (spherical_vox.cu:112-116
  // accumulates feat * (1/cnt) in an arbitrary atomic order; the oracle and
  // this kernel both use ascending point order)
  const int* perm = ws.perm + (size_t)b * n;
  const int* seg_off = ws.seg_off + (size_t)b * (n + 1);
  for (int si = tid; si < S; si += NT) {
    const int s = s_begin + si;
    const int off = seg_off[s], end = seg_off[s + 1];
    const float inv = pcr_inv_count(end - off);
    float acc[MG];
#pragma unroll
    for (int g = 0; g < MG; g++) acc[g] = 0.0f;
    for (int p = off; p < end; p++) {
      const int pt = perm[p];
#pragma unroll
      for (int g = 0; g < MG; g++)
        if (g < gcount) acc[g] = acc[g] + feat_s[(size_t)g * n + pt] * inv;
    }
#pragma unroll
    for (int g = 0; g < MG; g++)
      if (g < gcount) mean_s[(size_t)g * ns + si] = acc[g];
    scnt_s[si] = end - off;
  }
  if (tid < G) mean_s[(size_t)tid * ns + n] = 0.0f;
  if (tid == 0) scnt_s[n] = 0;
  __syncthreads();

  PCR_STAMP(10);
  // compact means for vox_stream_kernel (one tile per cloud: s_begin = 0)
  if (ws.means && ntiles == 1) {
    float* mo = ws.means + ((size_t)b * c + c0) * ws.ms;
    for (int g = 0; g < gcount; g++) {
      for (int si = tid; si < S; si += NT) mo[(size_t)g * ws.ms + si] = mean_s[(size_t)g * ns + si];
      if (tid == 0) mo[(size_t)g * ws.ms + n] = 0.0f;  // the empty-cell slot
    }
    if (grp == 0)
      for (int si = tid; si < S; si += NT)
        ws.segcnt[(size_t)b * ws.ms + si] = (unsigned short)scnt_s[si];
  }
  // stream the [gcount, cell0..cell1) slab once; zeros included
  float* ob = out + ((size_t)b * c + c0) * r3;
  int* cb = (cnt_out && grp == 0) ? cnt_out + (size_t)b * r3 : nullptr;
  // fused devox (role 3): each thread's PB points' corner data is loaded
  // before the streaming loop, and one point is devoxelised every few
  // streaming iterations, so the VALU / LDS work of the devox hides under the
  // outstanding grid stores instead of running after them
  constexpr int PB = 4;
  const bool interleave = role == 3 && (r3 & 3) == 0 && n <= PB * NT;
  float dv_w[PB][8];
  int dv_s[PB][8];
  float vmax[MG];
#pragma unroll
  for (int g = 0; g < MG; g++) vmax[g] = -__builtin_inff();
  auto devox_point = [&](int u) {
    const int i = tid + u * NT;
    if (i >= n) return;
    float* ov = devox + ((size_t)b * c + c0) * n;
#pragma unroll
    for (int g = 0; g < MG; g++) {
      if (g < gcount) {
        float fv[8];
#pragma unroll
        for (int q = 0; q < 8; q++) fv[q] = mean_s[(size_t)g * ns + dv_s[u][q]];
        const float v = pcr_wsum8(dv_w[u], fv);
        ov[(size_t)g * n + i] = v;
        vmax[g] = fmaxf(vmax[g], v);
      }
    }
  };
  if (interleave) {
    const float* Wt = dwgts + (size_t)b * 8 * n;
    const int* Dg = ws.dseg + (size_t)b * 8 * n;
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int i = tid + u * NT;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        dv_w[u][q] = i < n ? Wt[i + (size_t)q * n] : 0.0f;
        const int sg = i < n ? Dg[i + (size_t)q * n] : -1;
        dv_s[u][q] = sg >= 0 ? sg : n;  // empty corner -> the zero slot
      }
    }
  }
  // one streaming iteration: 4 consecutive cells from `base` (r^3 % 4 == 0),
  // one 16-byte store per channel (+ cnt).  The cells' ranks come from the
  // occupancy word and its prefix; a wave whose 256 cells are all empty
  // (common: the outer shells of the spherical grid) stores zeros directly.
  auto stream4 = [&](int base) {
    const int wl = (base >> 5) - wb;
    const unsigned word = bm_s[wl];
    const int sh = base & 31;
    const unsigned nib = (word >> sh) & 15u;
    if (__any(nib != 0u)) {
      const int pre = pre_s[wl] + __popc(word & ((1u << sh) - 1u));
      int ix[4];
      ix[0] = (nib & 1u) ? pre : n;
      ix[1] = (nib & 2u) ? pre + (int)(nib & 1u) : n;
      ix[2] = (nib & 4u) ? pre + __popc(nib & 3u) : n;
      ix[3] = (nib & 8u) ? pre + __popc(nib & 7u) : n;
#pragma unroll
      for (int g = 0; g < MG; g++) {
        if (g < gcount) {
          const float* ms = mean_s + (size_t)g * ns;
          const float4 v = {ms[ix[0]], ms[ix[1]], ms[ix[2]], ms[ix[3]]};
          *(float4*)(ob + (size_t)g * r3 + base) = v;
        }
      }
      if (cb) *(int4*)(cb + base) = int4{scnt_s[ix[0]], scnt_s[ix[1]], scnt_s[ix[2]], scnt_s[ix[3]]};
    } else {
      const float4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int g = 0; g < MG; g++)
        if (g < gcount) *(float4*)(ob + (size_t)g * r3 + base) = z;
      if (cb) *(int4*)(cb + base) = int4{0, 0, 0, 0};
    }
  };
  if (!(role & 1)) {
  } else if (interleave) {
    // the streaming iterations in PB chunks, one devox point after each
    const int iters = (cell1 - cell0 + NT * 4 - 1) / (NT * 4);
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int it1 = (u + 1) * iters / PB;
      for (int it = u * iters / PB; it < it1; it++) {
        const int base = cell0 + tid * 4 + it * NT * 4;
        if (base < cell1) stream4(base);
      }
      devox_point(u);
    }
  } else if ((r3 & 3) == 0) {
    for (int base = cell0 + tid * 4; base < cell1; base += NT * 4) stream4(base);
  } else {
    for (int cell = cell0 + tid; cell < cell1; cell += NT) {
      const int wl = (cell >> 5) - wb;
      const unsigned word = bm_s[wl];
      const unsigned bit = 1u << (cell & 31);
      const int rk = (word & bit) ? pre_s[wl] + __popc(word & (bit - 1u)) : -1;
      for (int g = 0; g < gcount; g++)
        ob[(size_t)g * r3 + cell] = rk >= 0 ? mean_s[(size_t)g * ns + rk] : 0.0f;
      if (cb) cb[cell] = rk >= 0 ? scnt_s[rk] : 0;
    }
  }

  PCR_STAMP(11);
  if (role & 2) {
    // spherical devoxelisation of this grid (spherical_trilinear_devox.cu:127-134)
    // evaluated from the LDS-resident means; requires one tile per cloud.
    // Corner -> segment map from prep (ws.dseg): the segment ids are the
    // rows of mean_s (one tile: s_begin = 0).  A dropped point has every
    // corner at -1 and zero weights, so its wsum8 is +0 like the
    // reference's untouched output.
    if (!interleave) {
      const float* Wt = dwgts + (size_t)b * 8 * n;
      const int* Dg = ws.dseg + (size_t)b * 8 * n;
      for (int i0 = 0; i0 < n; i0 += NT * PB) {
        // PB points per thread with all their corner loads in flight
#pragma unroll
        for (int u = 0; u < PB; u++) {
          const int i = i0 + tid + u * NT;
#pragma unroll
          for (int q = 0; q < 8; q++) {
            dv_w[u][q] = i < n ? Wt[i + (size_t)q * n] : 0.0f;
            const int sg = i < n ? Dg[i + (size_t)q * n] : -1;
            dv_s[u][q] = sg >= 0 ? sg : n;
          }
        }
        float* ov = devox + ((size_t)b * c + c0) * n;
#pragma unroll
        for (int u = 0; u < PB; u++) {
          const int i = i0 + tid + u * NT;
          if (i >= n) break;
#pragma unroll
          for (int g = 0; g < MG; g++) {
            if (g < gcount) {
              float fv[8];
#pragma unroll
              for (int q = 0; q < 8; q++)
                fv[q] = mean_s[(size_t)g * ns + dv_s[u][q]];
              const float v = pcr_wsum8(dv_w[u], fv);
              ov[(size_t)g * n + i] = v;
              vmax[g] = fmaxf(vmax[g], v);
            }
          }
        }
      }
    }
    if (desc) {
      __shared__ float red[NT / kWave][MG];
#pragma unroll
      for (int g = 0; g < MG; g++) {
        float m = wave_max(vmax[g]);
        if ((tid & 63) == 0) red[tid >> 6][g] = m;
      }
      lds_barrier();  // not waiting for the grid / devox stores
      if (tid < gcount) {
        float m = red[0][tid];
        for (int w = 1; w < NT / kWave; w++) m = fmaxf(m, red[w][tid]);
        desc[(size_t)b * c + c0 + tid] = m;
      }
    }
  }
  PCR_STAMP(12);
  }
}

// ------------------------------------------------------------ means kernel
// The first half of the split voxel stage: the voxel means of every occupied
// segment of G channels of one cloud, in ascending point order inside each
// voxel (the order vox_grid_kernel and the oracle use), written as compact
// rows ws.means[b][c][ms] (slot n = 0) + the segment counts (channel group
// 0), then the spherical devoxelisation of those means
// (spherical_trilinear_devox.cu:127-134, corner -> segment map from prep) and
// the per-cloud max-pooled descriptor.  Latency-bound by design (little
// work per workgroup), so every global read of the launch -- features,
// point order, segment offsets, corner segments and weights -- is requested
// before any is used: one round trip instead of a chain of dependent loads,
// which under the grid stream's write traffic take microseconds each.
constexpr int kMeansNT = 256;
constexpr int kMeansPB = 4;  // points per thread: clouds of <= 4 NT points
constexpr int kMeansMaxN = 2 * kMeansPB * kMeansNT;  // NT = 512 past 4 kMeansNT points (c3)
template <int G, int NT, bool DEVOX = true>
__global__ __launch_bounds__(NT) void vox_means_kernel(
    const float* __restrict__ feat, int c, int n, VoxWs ws, const float* __restrict__ dwgts,
    float* __restrict__ devox, float* __restrict__ desc, int ngrp) {
  constexpr int PB = kMeansPB;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so with
  // a batch of a multiple of 8 clouds XCD x runs every channel group of
  // clouds x, x + 8, ...: a cloud's corner data and point order (read by all
  // its channel groups) fill one XCD's L2 instead of all eight
  (void)PCR_PRIO(4);
  const int nb = gridDim.x / ngrp;
  const int b = (nb & 7) ? blockIdx.x / ngrp : (blockIdx.x & 7) + 8 * ((blockIdx.x >> 3) / ngrp);
  const int grp = (nb & 7) ? blockIdx.x % ngrp : (blockIdx.x >> 3) % ngrp;
  const int c0 = grp * G;
  const int gcount = min(G, c - c0);
  const int tid = threadIdx.x;
  const int ns = n + 1;
  float* feat_s = (float*)smem_raw;               // [G][n]
  float* mean_s = feat_s + (size_t)G * n;         // [G][ns], slot n = 0
  int* perm_s = (int*)(mean_s + (size_t)G * ns);  // [n]
  int* soff_s = perm_s + n;                       // [ns]

  // ---- every load in flight before any use
  const float* fb = feat + ((size_t)b * c + c0) * n;
  const int* gperm = ws.perm + (size_t)b * n;
  const int* gsoff = ws.seg_off + (size_t)b * (n + 1);
  float fv[G][PB];
  int pv[PB], sv[PB + 1];
#pragma unroll
  for (int e = 0; e < PB; e++) {
    const int i = e * NT + tid;
#pragma unroll
    for (int g = 0; g < G; g++) fv[g][e] = (i < n && g < gcount) ? fb[(size_t)g * n + i] : 0.0f;
    pv[e] = i < n ? gperm[i] : 0;
  }
#pragma unroll
  for (int e = 0; e <= PB; e++) {
    const int i = e * NT + tid;
    sv[e] = i <= n ? gsoff[i] : 0;
  }
  const float* Wt = dwgts + (size_t)b * 8 * n;
  const int* Dg = ws.dseg + (size_t)b * 8 * n;
  float dw[PB][8];
  int ds[PB][8];
#pragma unroll
  for (int e = 0; e < PB; e++) {
    const int i = e * NT + tid;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      dw[e][q] = (DEVOX && i < n) ? Wt[i + (size_t)q * n] : 0.0f;
      const int sg = (DEVOX && i < n) ? Dg[i + (size_t)q * n] : -1;
      ds[e][q] = sg >= 0 ? sg : n;  // empty corner -> the zero slot
    }
  }
  const int nseg = ws.nseg[b];
#pragma unroll
  for (int e = 0; e < PB; e++) {
    const int i = e * NT + tid;
    if (i < n) {
#pragma unroll
      for (int g = 0; g < G; g++) feat_s[(size_t)g * n + i] = fv[g][e];
      perm_s[i] = pv[e];
    }
  }
#pragma unroll
  for (int e = 0; e <= PB; e++) {
    const int i = e * NT + tid;
    if (i <= n) soff_s[i] = sv[e];
  }
  if (tid < G) mean_s[(size_t)tid * ns + n] = 0.0f;
  lds_barrier();

  // ---- means (spherical_vox.cu:112-116 order: ascending point ids; the
  // reference accumulates feat * (1/cnt) atomically in arbitrary order)
  float* mo = ws.means + ((size_t)b * c + c0) * ws.ms;
  for (int si = tid; si < nseg; si += NT) {
    const int off = soff_s[si], end = soff_s[si + 1];
    const float inv = pcr_inv_count(end - off);
    float acc[G];
#pragma unroll
    for (int g = 0; g < G; g++) acc[g] = 0.0f;
    for (int p = off; p < end; p++) {
      const int pt = perm_s[p];
#pragma unroll
      for (int g = 0; g < G; g++) acc[g] = acc[g] + feat_s[(size_t)g * n + pt] * inv;
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      mean_s[(size_t)g * ns + si] = acc[g];
      if (g < gcount) mo[(size_t)g * ws.ms + si] = acc[g];
    }
    if (grp == 0) ws.segcnt[(size_t)b * ws.ms + si] = (unsigned short)(end - off);
  }
  // the unused counts (slot n included) are 0, so the grid stream loads the
  // row as it stands
  if (grp == 0)
    for (int si = nseg + tid; si < ws.ms; si += NT) ws.segcnt[(size_t)b * ws.ms + si] = 0;
  if (tid < gcount) mo[(size_t)tid * ws.ms + n] = 0.0f;  // the empty-cell slot
  lds_barrier();

  // ---- devox of the G channels + descriptor (DEVOX = false: the grid
  // stream's DV role does it)
  if (!DEVOX) return;
  float vmax[G];
#pragma unroll
  for (int g = 0; g < G; g++) vmax[g] = -__builtin_inff();
  float* ov = devox + ((size_t)b * c + c0) * n;
#pragma unroll
  for (int e = 0; e < PB; e++) {
    const int i = e * NT + tid;
    if (i < n) {
#pragma unroll
      for (int g = 0; g < G; g++) {
        if (g < gcount) {
          float fq[8];
#pragma unroll
          for (int q = 0; q < 8; q++) fq[q] = mean_s[(size_t)g * ns + ds[e][q]];
          const float v = pcr_wsum8(dw[e], fq);
          ov[(size_t)g * n + i] = v;
          vmax[g] = fmaxf(vmax[g], v);
        }
      }
    }
  }
  if (desc) {
    __shared__ float red[NT / kWave][G];
#pragma unroll
    for (int g = 0; g < G; g++) {
      const float m = wave_max(vmax[g]);
      if ((tid & 63) == 0) red[tid >> 6][g] = m;
    }
    lds_barrier();  // not waiting for the devox / means stores
    if (tid < gcount) {
      float m = red[0][tid];
      for (int w = 1; w < NT / kWave; w++) m = fmaxf(m, red[w][tid]);
      desc[(size_t)b * c + c0 + tid] = m;
    }
  }
}

// ------------------------------------------------------- streaming kernel
// The dense [B, C, r^3] grid + cnt from the compact voxel means that the
// means / devox launch left in ws.means ([b][c][ms], one row per channel,
// occupied segments in voxel order, slot n = 0) and prep's occupancy bitmap.
// Small and persistent: per cloud a few workgroups, each a contiguous range
// of channel-pair items; ~35 KB of LDS and five waves, so the KNN
// selection's two workgroups fit on the same CU and run beside it (a dense
// write stream needs few waves; vox_grid_kernel's per-item setup is what
// made it occupy whole CUs).
//  - streamer waves (NS) only read LDS and store: they never wait on vmcnt,
//    so their stores stay in flight across items;
//  - the loader wave only loads: bitmap, word prefix and counts once, then
//    the means of item t+2 by LDS-DMA (global_load_lds_dwordx4) into the
//    third buffer while the streamers store item t.  Under the write stream
//    a load round trip takes microseconds; with two items of slack it never
//    holds a barrier.  The barriers wait for LDS operations only.
constexpr int kStreamG = 2;      // channels per item
constexpr int kStreamNG = 9;     // 1 KB LDS-DMA pieces per item: two rows of ms <= 1152 floats
constexpr int kStreamNB = 3;     // means buffers (item t streams, t+1 ready, t+2 landing)
constexpr int kStreamMaxN = 2048;  // two rows of ms <= 2052 floats: 17 pieces past 1024 points
constexpr int kStreamMaxW = 1024;  // occupancy words (r^3 <= 32768)

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
// DV (round 5): the streamer waves also evaluate the spherical devox of each
// item's channels from the means already in LDS (spherical_trilinear_devox.cu
// :127-134, vox_means_kernel's arithmetic: the same pcr_wsum8 of the same
// means) and the per-cloud descriptor max, so the means launch no longer
// reads the cloud's corner data once per channel pair: the corners of a
// streamer thread's points (n <= 1024: 1024 / NTS points) are loaded once per
// workgroup into registers.  Measured: the means launch without its devox ran
// the c2 step 382k -> 418k clouds/s (the same as with no means launch at all).
// clouds of <= 1024 points (c2): at 2048 points (c3) the role's 16 corner
// registers per point made the kernel 171 VGPRs and the c3 step 1.89 ->
// 1.95 ms (profiles/r05_ab_stream_devox.log), so c3 keeps the devox in the
// means launch
constexpr int kStreamDvMaxN = 1024;
// One streaming iteration of the grid-stream kernels: U groups of 4
// consecutive cells per thread, branch-free -- every LDS read of the U groups
// (occupancy word + prefix, then the means / counts, slot n = 0 for empty
// cells) is issued before any is waited on; one 16-byte store per channel
// (+ cnt) and group.  Stores with cache policy AUX (16 = sc1: write-through,
// the line is not kept in the XCD's L2, so the grid stream does not evict the
// other kernels' working sets).
template <int NTS, int U, int AUX, int G>
__device__ inline void stream_cells(int base0, float* ob, int gcount, const float* ms0, int* cb,
                                    int r3, int n, int ms, const unsigned* bm_s,
                                    const unsigned short* pre_s, const unsigned short* scnt_s) {
  unsigned word[U];
  int pw[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int base = min(base0 + u * NTS * 4, r3 - 4);
    word[u] = bm_s[base >> 5];
    pw[u] = pre_s[base >> 5];
  }
  int ix[U][4];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int sh = (base0 + u * NTS * 4) & 31;
    const unsigned nib = (word[u] >> sh) & 15u;
    const int pre = pw[u] + __popc(word[u] & ((1u << sh) - 1u));
    ix[u][0] = (nib & 1u) ? pre : n;
    ix[u][1] = (nib & 2u) ? pre + (int)(nib & 1u) : n;
    ix[u][2] = (nib & 4u) ? pre + __popc(nib & 3u) : n;
    ix[u][3] = (nib & 8u) ? pre + __popc(nib & 7u) : n;
  }
  float4 v[U][G];
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int g = 0; g < G; g++) {
      if (g < gcount) {
        const float* ms_g = ms0 + (size_t)g * ms;
        v[u][g] = float4{ms_g[ix[u][0]], ms_g[ix[u][1]], ms_g[ix[u][2]], ms_g[ix[u][3]]};
      }
    }
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(ob, (short)0, G * r3 * 4, 0x00020000);
#pragma unroll
  for (int g = 0; g < G; g++) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int base = base0 + u * NTS * 4;
      if (base < r3 && g < gcount)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v[u][g]), rs,
                                               (g * r3 + base) * 4, 0, AUX);
    }
  }
  if (cb) {
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(cb, (short)0, r3 * 4, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int base = base0 + u * NTS * 4;
      const u32x4_t cv = {scnt_s[ix[u][0]], scnt_s[ix[u][1]], scnt_s[ix[u][2]], scnt_s[ix[u][3]]};
      if (base < r3) __builtin_amdgcn_raw_buffer_store_b128(cv, rc, base * 4, 0, AUX);
    }
  }
}

// DVN: 0 = no devox role; else the most points per cloud
template <int NS, int NB, int U, int AUX, int G = kStreamG, int NG = kStreamNG, int DVN = 0>
__global__ __launch_bounds__((NS + 1) * 64) void vox_stream_kernel(int c, int n, int r3, VoxWs ws,
                                                                  float* __restrict__ out,
                                                                  int* __restrict__ cnt_out,
                                                                  int ngrp, int wpc, int per,
                                                                  const float* __restrict__ dwgts,
                                                                  float* __restrict__ devox,
                                                                  float* __restrict__ desc) {
  constexpr int D = NB - 1;     // prefetch distance in items
  constexpr int NTS = NS * 64;  // streamer threads
  constexpr int BUFB = NG * 1024;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int W = ws.W;
  const int ms = ws.ms;
  float* mean_s = (float*)smem_raw;                                // [NB][BUFB / 4]
  unsigned* bm_s = (unsigned*)(smem_raw + NB * BUFB);              // [W]
  unsigned short* pre_s = (unsigned short*)(bm_s + W);             // [W -> 256 B]
  unsigned short* scnt_s = pre_s + (W + 127) / 128 * 128;          // [ms -> 256 B], slot n = 0
  (void)PCR_PRIO(5);
  const int b = blockIdx.x / wpc;
  const int j0 = (blockIdx.x % wpc) * per;
  const int nit = min(ngrp, j0 + per) - j0;
  if (nit <= 0) return;  // uniform over the workgroup
  const int tid = threadIdx.x;
  const int lt = tid & 63;
  PCR_STAMP(0);

  if (tid >= NTS) {
    // ---- loader wave
    // item j (channel pair) of this cloud into means buffer `buf`: NG whole
    // 1 KB pieces (the two rows are adjacent; the tail past them is unused)
    auto issue = [&](int j, int buf) {
      const char* src = (const char*)(ws.means + ((size_t)b * c + (size_t)j * G) * ms);
      char* dst = (char*)smem_raw + buf * BUFB;
#pragma unroll
      for (int p = 0; p < NG; p++)
        __builtin_amdgcn_global_load_lds((gbl_void_p)(src + p * 1024 + lt * 16),
                                         (lds_void_p)(dst + p * 1024), 16, 0, 0);
    };
    // every load of the prologue in flight at once: the first two items'
    // means, the bitmap, the segment counts and nseg
#ifdef PCR_DIAG
    if (tid == NTS && PCR_WG_LINEAR < 1024) pcr_diag_stamps[PCR_WG_LINEAR][6] = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
    for (int q = 0; q < D; q++)
      if (q < nit) issue(j0 + q, q);
    {
      // bitmap, its word prefix (prep's) and the segment counts (the means
      // launch's, unused slots 0) by LDS-DMA too (4-byte pieces: 256 B per
      // wave instruction), so the loader holds no staging registers and
      // computes nothing before the first barrier (round 6: the word prefix
      // was scanned here, 4 us of the launch's 8 us prologue)
      auto dma4 = [&](void* dst, const void* src, int nbytes) {
        for (int p = 0; p * 256 < nbytes; p++)
          __builtin_amdgcn_global_load_lds((gbl_void_p)((const char*)src + p * 256 + lt * 4),
                                           (lds_void_p)((char*)dst + p * 256), 4, 0, 0);
      };
      dma4(bm_s, ws.bitmap + (size_t)b * W, W * 4);
      dma4(pre_s, ws.wpre16 + (size_t)b * W, W * 2);
      dma4(scnt_s, ws.segcnt + (size_t)b * ms, ms * 2);
    }
    wait_vmcnt<0>();
#ifdef PCR_DIAG
    if (tid == NTS && PCR_WG_LINEAR < 1024) pcr_diag_stamps[PCR_WG_LINEAR][7] = __builtin_amdgcn_s_memtime();
#endif
    lds_only_barrier();
    for (int it = 0; it < nit; it++) {
      // buffer (it + D) % NB held item it - 1, released by the last barrier;
      // item it + 1 must have landed before the streamers start it
      if (it + D < nit) {
        issue(j0 + it + D, (it + D) % NB);
        wait_vmcnt<NG * (D - 1)>();
      } else {
        wait_vmcnt<0>();
      }
      lds_only_barrier();
    }
    return;
  }

  // ---- streamer waves
  // DV: this thread's points i = tid + e NTS, their 8 corners' segments
  // (empty corner -> slot n, whose mean is 0; two u16 per register, prep's
  // packed map: one 16-byte load per point) and weights, for every item.
  // Issued after the first barrier (the loader's prologue loads go first)
  // and waited for only at the first item's devox (round 6: the packing used
  // to wait for them before the first barrier, so the launch's first grid
  // stores waited behind 16 MB of corner loads)
  constexpr bool DV = DVN > 0;
  constexpr int PBS = DV ? DVN / NTS : 1;
  lds_only_barrier();
  unsigned dsg[PBS][4];
  float dwt[PBS][8];
  __shared__ float dred_s[2][DV ? NS : 1][G];  // per-wave descriptor partials, by item parity
  if (DV) {
    const float* Wt = dwgts + (size_t)b * 8 * n;
    const uint4* Dg = (const uint4*)(ws.dseg16 + (size_t)b * n * 4);
#pragma unroll
    for (int e = 0; e < PBS; e++) {
      const int i = e * NTS + tid;
      const uint4 v = i < n ? Dg[i] : uint4{0u, 0u, 0u, 0u};
      dsg[e][0] = v.x;
      dsg[e][1] = v.y;
      dsg[e][2] = v.z;
      dsg[e][3] = v.w;
#pragma unroll
      for (int q = 0; q < 8; q++) dwt[e][q] = i < n ? Wt[i + (size_t)q * n] : 0.0f;
    }
  }
  PCR_STAMP(1);
  // the sweep starts at a workgroup-dependent step of the item and wraps, so
  // the workgroups do not all hit the same HBM channels at once
  const int nstep = (r3 + NTS * 4 * U - 1) / (NTS * 4 * U);
  const int rot = (int)(blockIdx.x % nstep);
  for (int it = 0; it < nit; it++) {
    const int j = j0 + it;
    const int c0 = j * G;
    const int gcount = min(G, c - c0);
    float* ob = out + ((size_t)b * c + c0) * r3;
    int* cb = (cnt_out && j == 0) ? cnt_out + (size_t)b * r3 : nullptr;
    const float* ms0 = mean_s + (size_t)(it % NB) * (BUFB / 4);
    for (int st = 0; st < nstep; st++) {
      const int sp = st + rot < nstep ? st + rot : st + rot - nstep;
      stream_cells<NTS, U, AUX, G>(sp * NTS * 4 * U + tid * 4, ob, gcount, ms0, cb, r3, n, ms,
                                   bm_s, pre_s, scnt_s);
    }
    if (it < 4) PCR_STAMP(12 + it);
    if (DV) {
      // devox of the item's channels (vox_means_kernel's loop) + descriptor partials
      float vmax[G];
#pragma unroll
      for (int g = 0; g < G; g++) vmax[g] = -__builtin_inff();
      float* ov = devox + ((size_t)b * c + c0) * n;
#pragma unroll
      for (int e = 0; e < PBS; e++) {
        const int i = e * NTS + tid;
        if (i < n) {
#pragma unroll
          for (int g = 0; g < G; g++) {
            if (g < gcount) {
              float fq[8];
#pragma unroll
              for (int q = 0; q < 8; q++)
                fq[q] = ms0[(size_t)g * ms + ((dsg[e][q >> 1] >> (16 * (q & 1))) & 0xFFFFu)];
              const float v = pcr_wsum8(dwt[e], fq);
              ov[(size_t)g * n + i] = v;
              vmax[g] = fmaxf(vmax[g], v);
            }
          }
        }
      }
      if (desc) {
#pragma unroll
        for (int g = 0; g < G; g++) {
          const float m = wave_max(vmax[g]);
          if (lt == 0) dred_s[it & 1][tid >> 6][g] = m;
        }
      }
    }
    if (it < 4) PCR_STAMP(2 + it);
    lds_only_barrier();
    if (it < 4) PCR_STAMP(8 + it);
    if (DV && desc && tid < gcount) {
      // (dred_s[it & 1] is rewritten two items later, after the next barrier)
      float m = dred_s[it & 1][0][tid];
#pragma unroll
      for (int w = 1; w < NS; w++) m = fmaxf(m, dred_s[it & 1][w][tid]);
      desc[(size_t)b * c + c0 + tid] = m;
    }
  }
}

// LDS of vox_stream_kernel: kStreamNB means buffers of NGP KB, the bitmap,
// its u16 word prefix and the u16 segment counts (each in whole 256-byte
// LDS-DMA pieces)
static size_t stream_smem_bytes(int NGP, int W, int ms) {
  return (size_t)kStreamNB * NGP * 1024 + (size_t)W * 4 + ((size_t)W * 2 + 255) / 256 * 256 +
         ((size_t)ms * 2 + 255) / 256 * 256;
}

// ------------------------------------------------------ backward gather
// grad_x[b,j,i] = grad_y[b,j,ind[i]] * (1/cnt)  (spherical_vox.cu:151-162)
// One thread per point and kGradCG channels: the point's voxel and count are
// loaded once and all kGradCG gathers are issued before any is used (a
// runtime-length channel loop waited for each gather in turn: a chain of
// dependent HBM round trips per thread).
constexpr int kGradCG = 16;
__global__ __launch_bounds__(256) void avg_vox_grad_kernel(const float* __restrict__ grad_y,
                                                           const int* __restrict__ ind,
                                                           const int* __restrict__ cnt, int c,
                                                           int n, int r3,
                                                           float* __restrict__ grad_x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.z;
  const int j0 = blockIdx.y * kGradCG;
  if (i >= n) return;
  const int pos = ind[(size_t)b * n + i];
  float inv = 0.0f;
  bool ok = pos >= 0 && pos < r3;
  if (ok) {
    const int ct = cnt[(size_t)b * r3 + pos];
    ok = ct > 0;
    if (ok) inv = pcr_inv_count(ct);
  }
  const int jn = min(kGradCG, c - j0);
  const float* gy = grad_y + ((size_t)b * c + j0) * r3 + (ok ? pos : 0);
  float v[kGradCG];
#pragma unroll
  for (int j = 0; j < kGradCG; j++) v[j] = (ok && j < jn) ? gy[(size_t)j * r3] : 0.0f;
  float* gx = grad_x + ((size_t)b * c + j0) * n + i;
#pragma unroll
  for (int j = 0; j < kGradCG; j++)
    if (j < jn) gx[(size_t)j * n] = v[j] * inv;
}

// The same gather for clouds of <= 2048 points, in voxel-row order: one
// workgroup of 1024 threads per (cloud, kGradSortCG channels) counting-sorts
// its points by 32-voxel row (ind >> 5, one 128-byte line of a channel's
// gradient row) in LDS, so each wave's gathers of a channel fall in a few
// lines instead of 64 (a point-order wave touches ~64 lines of a 128 KB row:
// the kernel above is bound by that request rate, 0.49 ms at the c3 shape);
// the values go to LDS at the points' original positions and leave as
// coalesced rows.  Each output is the same single product as above, in any
// order, so the same bits.
constexpr int kGradSortThreads = 1024;
constexpr int kGradSortMaxN = 2048;
constexpr int kGradSortCG = 16;  // channels per workgroup
constexpr int kGradSortU = 4;    // channels gathered per pass
constexpr int kGradSortMaxRows = 8192;
__global__ __launch_bounds__(kGradSortThreads) void avg_vox_grad_sorted_kernel(
    const float* __restrict__ grad_y, const int* __restrict__ ind, const int* __restrict__ cnt,
    int c, int n, int r3, float* __restrict__ grad_x) {
  constexpr int PT = kGradSortMaxN / kGradSortThreads;  // points per thread
  // row counters (then starts), reused as the output staging rows
  __shared__ int un_s[kGradSortU * kGradSortMaxN > kGradSortMaxRows + 1
                          ? kGradSortU * kGradSortMaxN : kGradSortMaxRows + 1];
  __shared__ int spos_s[kGradSortMaxN];              // voxel of sorted point s (0 if dropped)
  __shared__ float sinv_s[kGradSortMaxN];            // 1 / count of its voxel (0 if dropped)
  __shared__ unsigned short sidx_s[kGradSortMaxN];   // its original index
  __shared__ int scan_s[kGradSortThreads / kWave + 1];
  int* cnt_s = un_s;
  float* out_s = (float*)un_s;
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * kGradSortCG;
  const int cn = min(kGradSortCG, c - c0);
  const int tid = threadIdx.x;
  const int rows = (r3 + 31) >> 5;  // + 1: the bin of dropped points
  for (int t = tid; t <= rows; t += kGradSortThreads) cnt_s[t] = 0;
  lds_only_barrier();
  int key[PT], slot[PT], pos[PT];
  float inv[PT];
#pragma unroll
  for (int u = 0; u < PT; u++) {
    const int i = u * kGradSortThreads + tid;
    key[u] = -1;
    if (i < n) {
      int p = ind[(size_t)b * n + i];
      bool ok = p >= 0 && p < r3;
      float iv = 0.0f;
      if (ok) {
        const int ct = cnt[(size_t)b * r3 + p];
        ok = ct > 0;
        if (ok) iv = pcr_inv_count(ct);
      }
      pos[u] = ok ? p : 0;
      inv[u] = iv;
      key[u] = ok ? (p >> 5) : rows;
      slot[u] = atomicAdd(&cnt_s[key[u]], 1);
    }
  }
  lds_only_barrier();
  // exclusive scan of rows + 1 counters, kGradSortMaxRows / 1024 + 1 per thread
  {
    constexpr int CPT = (kGradSortMaxRows + 1 + kGradSortThreads - 1) / kGradSortThreads;
    int v[CPT], sum = 0;
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      const int rr = tid * CPT + q;
      v[q] = rr <= rows ? cnt_s[rr] : 0;
      sum += v[q];
    }
    int run = block_inclusive_scan(sum, scan_s) - sum;
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      const int rr = tid * CPT + q;
      if (rr <= rows) cnt_s[rr] = run;
      run += v[q];
    }
  }
  lds_only_barrier();
#pragma unroll
  for (int u = 0; u < PT; u++) {
    if (key[u] >= 0) {
      const int s2 = cnt_s[key[u]] + slot[u];
      spos_s[s2] = pos[u];
      sinv_s[s2] = inv[u];
      sidx_s[s2] = (unsigned short)(u * kGradSortThreads + tid);
    }
  }
  lds_only_barrier();  // counters dead: un_s becomes the output rows
  for (int j0 = 0; j0 < cn; j0 += kGradSortU) {
    const int jn = min(kGradSortU, cn - j0);
    const float* gy = grad_y + ((size_t)b * c + c0 + j0) * r3;
    float v[PT][kGradSortU];
#pragma unroll
    for (int u = 0; u < PT; u++) {
      const int s2 = u * kGradSortThreads + tid;
      const int p = s2 < n ? spos_s[s2] : 0;
#pragma unroll
      for (int q = 0; q < kGradSortU; q++) v[u][q] = (s2 < n && q < jn) ? gy[(size_t)q * r3 + p] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < PT; u++) {
      const int s2 = u * kGradSortThreads + tid;
      if (s2 < n) {
        // iv == 0 marks a dropped point: +0 as the reference leaves it
        // (spherical_vox.cu:153-156), not grad_y[voxel 0] * 0 (-0 / NaN)
        const float iv = sinv_s[s2];
        const int i = sidx_s[s2];
#pragma unroll
        for (int q = 0; q < kGradSortU; q++)
          out_s[q * kGradSortMaxN + i] = iv != 0.0f ? v[u][q] * iv : 0.0f;
      }
    }
    lds_only_barrier();
    float* gx = grad_x + ((size_t)b * c + c0 + j0) * n;
#pragma unroll
    for (int q = 0; q < kGradSortU; q++) {
      if (q < jn) {
#pragma unroll
        for (int u = 0; u < PT; u++) {
          const int i = u * kGradSortThreads + tid;
          if (i < n) gx[(size_t)q * n + i] = out_s[q * kGradSortMaxN + i];
        }
      }
    }
    lds_only_barrier();  // rows read before the next pass writes them
  }
}

// ------------------------------------------------------ normalize only
__global__ __launch_bounds__(kPrepThreads) void sph_normalize_kernel(
    const float* __restrict__ coords, int n, int E, float* __restrict__ out) {
  __shared__ double red[48];
  __shared__ float s_stat[4];
  __shared__ float wm[kPrepThreads / kWave];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* x = coords + (size_t)b * 3 * n;
  float* o = out + (size_t)b * 3 * n;
  float px[kMaxE], py[kMaxE], pz[kMaxE];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int i = e * kPrepThreads + tid;
    const bool ok = e < E && i < n;
    px[e] = ok ? x[i] : 0.0f;
    py[e] = ok ? x[i + n] : 0.0f;
    pz[e] = ok ? x[i + 2 * n] : 0.0f;
  }
  cloud_mean<kPrepThreads>(px, py, pz, E, n, red, s_stat);
  const float m0 = s_stat[0], m1 = s_stat[1], m2 = s_stat[2];
  float mx = 0.0f;
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    if (e < E && e * kPrepThreads + tid < n) {
      px[e] -= m0;
      py[e] -= m1;
      pz[e] -= m2;
      mx = fmaxf(mx, __builtin_sqrtf(pcr_sumsq3f(px[e], py[e], pz[e])));
    }
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) wm[tid >> 6] = mx;
  __syncthreads();
  if (tid == 0) {
    float m = 0.0f;
    for (int w = 0; w < kPrepThreads / kWave; w++) m = fmaxf(m, wm[w]);
    s_stat[3] = m + 1e-20f;
  }
  __syncthreads();
  const float den = s_stat[3];
#pragma unroll
  for (int e = 0; e < kMaxE; e++) {
    const int i = e * kPrepThreads + tid;
    if (e < E && i < n) {
      o[i] = px[e] / den;
      o[i + n] = py[e] / den;
      o[i + 2 * n] = pz[e] / den;
    }
  }
}

// ------------------------------------------------- clouds of > 4096 points
// A stable counting sort by voxel, hand-written, at any size: (1) per-point
// voxel index and count atomics, whose return value is the point's arrival
// slot in its voxel; (2) a per-cloud exclusive scan of the counts (tile sums,
// then each tile scans itself after the sum of the tiles before it) locates
// every voxel's segment; (3) each point lands at start + slot (arrival
// order); (4) each point of a segment of 1 < m <= 64 takes its rank by point
// id among the segment (m reads), a larger segment is sorted by a stable
// workgroup radix sort, so every voxel's points end up in ascending point
// order -- the order the oracle sums in; (5) one thread per voxel sums
// its segment in that order and writes all C channels, so the dense grid is
// written once, coalesced, zeros included.  The reference scatters C fp32
// atomics per point (spherical_vox.cu:103-123, one cache line each).
struct BigVoxWs {
  int* slot;      // [b][n] arrival slot of each point in its voxel
  int* perm_u;    // [b][n] points by voxel, arrival order within a voxel
  int* perm;      // [b][n] points by voxel, ascending within a voxel
  int* start;     // [b][r3] segment start of each voxel (relative to its cloud)
  int* tsum;      // [b][ntile] counts per scan tile
  int* big;       // [1 + b n / (kRankScan + 1)]: count, then voxels of > kRankScan points
  float* featT;   // [b][n][c] point-major copy of the features (nullptr: c == 0)
  int ntile;
};

// segments of up to this many points take their rank by a scan of the
// segment (m reads per point); larger ones are sorted by vox_seg_sort_kernel
constexpr int kRankScan = 64;

constexpr int kBigScanThreads = 256;
constexpr int kBigScanPer = 16;
constexpr int kBigScanTile = kBigScanThreads * kBigScanPer;

static size_t big_ws_layout(int b, int n, int r, BigVoxWs* ws, void* base, int c = 0) {
  const int64_t r3 = (int64_t)r * r * r;
  const size_t nk = (size_t)b * n, nr = (size_t)b * r3;
  const int ntile = (int)((r3 + kBigScanTile - 1) / kBigScanTile);
  size_t off = 0;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off = align_up(off + bytes, 256);
    return q;
  };
  int* slot = (int*)take(nk * 4);
  int* perm_u = (int*)take(nk * 4);
  int* perm = (int*)take(nk * 4);
  int* start = (int*)take(nr * 4);
  int* tsum = (int*)take((size_t)b * ntile * 4);
  int* big = (int*)take((1 + nk / (kRankScan + 1)) * 4);
  float* ft = c > 0 ? (float*)take(nk * (size_t)c * 4) : nullptr;
  if (ws) {
    ws->slot = slot;
    ws->perm_u = perm_u;
    ws->perm = perm;
    ws->start = start;
    ws->tsum = tsum;
    ws->big = big;
    ws->featT = ft;
    ws->ntile = ntile;
  }
  return off;
}

template <int MODE>
__global__ __launch_bounds__(256) void vox_key_big_kernel(const float* __restrict__ coords_f,
                                                          const int* __restrict__ coords_i, int n,
                                                          int r, int* __restrict__ ind,
                                                          int* __restrict__ cnt,
                                                          int* __restrict__ slot) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= n) return;
  const int r3 = r * r * r;
  int v;
  bool valid;
  if (MODE == kCube) {
    const int* x = coords_i + (size_t)b * 3 * n;
    v = x[i] * r * r + x[i + n] * r + x[i + 2 * n];
    valid = v >= 0 && v < r3;
  } else {
    const float* x = coords_f + (size_t)b * 3 * n;
    v = pcr_sph_index(x[i], x[i + n], x[i + 2 * n], r);
    valid = v >= 0;
  }
  ind[(size_t)b * n + i] = v;
  slot[(size_t)b * n + i] = valid ? atomicAdd(&cnt[(size_t)b * r3 + v], 1) : -1;
}

// per-cloud exclusive scan of the voxel counts, pass 1: each tile's total
__global__ __launch_bounds__(kBigScanThreads) void vox_scan_tiles_kernel(
    const int* __restrict__ cnt, int r3, int ntile, int* __restrict__ tsum) {
  __shared__ int red[kBigScanThreads / kWave];
  const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int* C = cnt + (size_t)b * r3 + (size_t)t * kBigScanTile;
  const int lim = min(kBigScanTile, r3 - t * kBigScanTile);
  int s = 0;
#pragma unroll
  for (int e = 0; e < kBigScanPer; e++) {
    const int v = e * kBigScanThreads + tid;
    s += v < lim ? C[v] : 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < kBigScanThreads / kWave; w++) tot += red[w];
    tsum[(size_t)b * ntile + t] = tot;
  }
}

// pass 2: each tile adds the totals of the tiles before it (in order) and
// scans its counts; thread t owns kBigScanPer consecutive voxels
__global__ __launch_bounds__(kBigScanThreads) void vox_scan_apply_kernel(
    const int* __restrict__ cnt, int r3, int ntile, const int* __restrict__ tsum,
    int* __restrict__ start) {
  __shared__ int scan_s[kBigScanThreads / kWave + 1];
  __shared__ int base_s;
  const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  if (tid < 64) {
    int s = 0;
    for (int q = tid; q < t; q += 64) s += tsum[(size_t)b * ntile + q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
    if (tid == 0) base_s = s;
  }
  const int v0 = t * kBigScanTile + tid * kBigScanPer;
  const int* C = cnt + (size_t)b * r3;
  int c[kBigScanPer], sum = 0;
#pragma unroll
  for (int e = 0; e < kBigScanPer; e++) {
    c[e] = v0 + e < r3 ? C[v0 + e] : 0;
    sum += c[e];
  }
  const int incl = block_inclusive_scan(sum, scan_s);  // its barriers also publish base_s
  int run = base_s + incl - sum;
  int* S = start + (size_t)b * r3;
#pragma unroll
  for (int e = 0; e < kBigScanPer; e++) {
    if (v0 + e < r3) S[v0 + e] = run;
    run += c[e];
  }
}

// every point at its voxel's start + arrival slot
__global__ __launch_bounds__(256) void vox_place_big_kernel(const int* __restrict__ ind,
                                                            const int* __restrict__ slot, int n,
                                                            int r3, const int* __restrict__ start,
                                                            int* __restrict__ perm_u) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= n) return;
  const int sl = slot[(size_t)b * n + i];
  if (sl < 0) return;
  const int v = ind[(size_t)b * n + i];
  perm_u[(size_t)b * n + start[(size_t)b * r3 + v] + sl] = i;
}

// every point's final place: its rank by point id within its voxel's segment
// (m reads for a voxel of m <= kRankScan points; one-point voxels copy).  A
// larger segment (duplicated points, a cloud padded by repeating a point) is
// listed once, by its first arrival, for vox_seg_sort_kernel: the scan would
// cost m^2 reads there.
__global__ __launch_bounds__(256) void vox_rank_big_kernel(const int* __restrict__ ind,
                                                           const int* __restrict__ slot, int n,
                                                           int r3, const int* __restrict__ cnt,
                                                           const int* __restrict__ start,
                                                           const int* __restrict__ perm_u,
                                                           int* __restrict__ perm,
                                                           int* __restrict__ big) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= n) return;
  const int sl = slot[(size_t)b * n + i];
  if (sl < 0) return;
  const int v = ind[(size_t)b * n + i];
  const size_t vi = (size_t)b * r3 + v;
  const int m = cnt[vi];
  if (m > kRankScan) {
    if (sl == 0) big[1 + atomicAdd(&big[0], 1)] = (int)vi;
    return;
  }
  const int* seg = perm_u + (size_t)b * n + start[vi];
  int rank = 0;
  for (int x = 0; x < m; x++) rank += seg[x] < i ? 1 : 0;
  perm[(size_t)b * n + start[vi] + rank] = i;
}

// the listed large segments: one workgroup per segment (grid-stride over the
// list), its point ids sorted ascending by a stable workgroup radix sort
// (O(m) per 8-bit pass) from the arrival order (perm_u) into perm
constexpr int kSegSortThreads = 1024;
__global__ __launch_bounds__(kSegSortThreads) void vox_seg_sort_kernel(
    const int* __restrict__ big, const int* __restrict__ cnt, const int* __restrict__ start,
    int n, int r3, int kbits, int* __restrict__ perm_u, int* __restrict__ perm) {
  __shared__ int rs_lds[(2 + kSegSortThreads / kWave) * 256];
  const int nb = big[0];
  for (int e = blockIdx.x; e < nb; e += gridDim.x) {
    const int vi = big[1 + e];
    const int m = cnt[vi];
    const size_t off = (size_t)(vi / r3) * n + start[vi];
    int* res = wg_radix_sort<kSegSortThreads>(perm_u + off, perm + off, m, kbits,
                                              [](int v) { return v; }, rs_lds);
    if (res != perm + off)
      for (int t = threadIdx.x; t < m; t += kSegSortThreads) perm[off + t] = res[t];
    __syncthreads();
  }
}

// the listed large segments' means: one workgroup per segment (grid-stride
// over the list), a thread per channel summing the segment's points in
// ascending order (the order of the thread-per-voxel kernels, which skip
// these voxels), eight point ids and their values loaded ahead of the sums.
// FT: point-major features [b][n][c] (else channel-major [b][c][n]).
template <bool FT>
__global__ __launch_bounds__(256) void vox_seg_gather_kernel(
    const int* __restrict__ big, const float* __restrict__ feat, const int* __restrict__ cnt,
    const int* __restrict__ start, const int* __restrict__ perm, int c, int n, int r3,
    float* __restrict__ out) {
  constexpr int kB = 8;
  const int nb = big[0];
  for (int e = blockIdx.x; e < nb; e += gridDim.x) {
    const int vi = big[1 + e];
    const int b = vi / r3, v = vi - b * r3;
    const int m = cnt[vi];
    const int* P = perm + (size_t)b * n + start[vi];
    const float inv = pcr_inv_count(m);
    for (int ch = threadIdx.x; ch < c; ch += blockDim.x) {
      auto val = [&](int i) {
        return FT ? feat[((size_t)b * n + i) * c + ch] : feat[((size_t)b * c + ch) * n + i];
      };
      float acc = 0.0f;
      int s = 0;
      for (; s + kB <= m; s += kB) {
        int pi[kB];
        float x[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) pi[u] = P[s + u];
#pragma unroll
        for (int u = 0; u < kB; u++) x[u] = val(pi[u]);
#pragma unroll
        for (int u = 0; u < kB; u++) acc += x[u] * inv;
      }
      for (; s < m; s++) acc += val(P[s]) * inv;
      __builtin_nontemporal_store(acc, &out[((size_t)b * c + ch) * r3 + v]);
    }
  }
}

// one thread per voxel: its segment of the sorted points, summed per channel
// in ascending point order (acc += f * inv, the product rounded first)
__global__ __launch_bounds__(256) void vox_gather_big_kernel(
    const float* __restrict__ feat, const int* __restrict__ cnt, const int* __restrict__ start,
    const int* __restrict__ perm, int c, int n, int r3, float* __restrict__ out) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (v >= r3) return;
  const size_t vi = (size_t)b * r3 + v;
  const int m = cnt[vi];
  if (m > kRankScan) return;  // vox_seg_gather_kernel
  const int* P = perm + (size_t)b * n + start[vi];
  const float* F = feat + (size_t)b * c * n;
  float* O = out + (size_t)b * c * r3 + v;
  if (m == 0) {
    for (int ch = 0; ch < c; ch++) O[(size_t)ch * r3] = 0.0f;
    return;
  }
  const float inv = pcr_inv_count(m);
  constexpr int kHold = 8;
  int pts[kHold];
#pragma unroll
  for (int s = 0; s < kHold; s++) pts[s] = s < m ? P[s] : 0;
  for (int ch = 0; ch < c; ch++) {
    const float* f = F + (size_t)ch * n;
    float acc = 0.0f;
#pragma unroll
    for (int s = 0; s < kHold; s++)
      if (s < m) acc += f[pts[s]] * inv;
    for (int s = kHold; s < m; s++) acc += f[P[s]] * inv;
    O[(size_t)ch * r3] = acc;
  }
}

// Fixed-order normalisation for any n (same order as cloud_mean: thread t
// sums points t, t + 1024, ... ascending in double; wave halving trees).
__global__ __launch_bounds__(kPrepThreads) void sph_normalize_big_kernel(
    const float* __restrict__ coords, int n, float* __restrict__ out) {
  __shared__ double red[48];
  __shared__ float s_stat[4];
  __shared__ float wm[kPrepThreads / kWave];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* x = coords + (size_t)b * 3 * n;
  float* o = out + (size_t)b * 3 * n;
  double s[3] = {0.0, 0.0, 0.0};
  for (int i = tid; i < n; i += kPrepThreads) {
    s[0] += (double)x[i];
    s[1] += (double)x[i + n];
    s[2] += (double)x[i + 2 * n];
  }
#pragma unroll
  for (int a = 0; a < 3; a++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double v = __shfl_down(s[a], off, kWave);
      if (lane < off) s[a] += v;
    }
    if (lane == 0) red[a * 16 + w] = s[a];
  }
  __syncthreads();
  if (tid < 3) {
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = red[tid * 16 + i];
#pragma unroll
    for (int off = 8; off > 0; off >>= 1)
#pragma unroll
      for (int i = 0; i < off; i++) v[i] += v[i + off];
    s_stat[tid] = (float)(v[0] / (double)n);
  }
  __syncthreads();
  const float m0 = s_stat[0], m1 = s_stat[1], m2 = s_stat[2];
  float mx = 0.0f;
  for (int i = tid; i < n; i += kPrepThreads)
    mx = fmaxf(mx, __builtin_sqrtf(pcr_sumsq3f(x[i] - m0, x[i + n] - m1, x[i + 2 * n] - m2)));
  mx = wave_max(mx);
  if (lane == 0) wm[w] = mx;
  __syncthreads();
  if (tid == 0) {
    float m = 0.0f;
    for (int k = 0; k < kPrepThreads / kWave; k++) m = fmaxf(m, wm[k]);
    s_stat[3] = m + 1e-20f;
  }
  __syncthreads();
  const float den = s_stat[3];
  for (int i = tid; i < n; i += kPrepThreads) {
    o[i] = (x[i] - m0) / den;
    o[i + n] = (x[i + n] - m1) / den;
    o[i + 2 * n] = (x[i + 2 * n] - m2) / den;
  }
}

// [c][n] -> [n][c] per cloud through a 64 x 64 LDS tile (coalesced both ways)
__global__ __launch_bounds__(256) void feat_transpose_kernel(const float* __restrict__ feat,
                                                             int c, int n,
                                                             float* __restrict__ featT) {
  __shared__ float t[64][65];
  const int b = blockIdx.z, n0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const float* F = feat + (size_t)b * c * n;
  float* T = featT + (size_t)b * n * c;
  for (int y = ty; y < 64; y += 4)
    if (c0 + y < c && n0 + tx < n) t[y][tx] = F[(size_t)(c0 + y) * n + n0 + tx];
  __syncthreads();
  for (int y = ty; y < 64; y += 4)
    if (n0 + y < n && c0 + tx < c) T[(size_t)(n0 + y) * c + c0 + tx] = t[tx][y];
}

// vox_gather_big_kernel on the point-major copy: a voxel's point reads 16
// consecutive channels (64 B) at a time instead of 16 scattered lines
template <int CH>
__global__ __launch_bounds__(256) void vox_gather_big_t_kernel(
    const float* __restrict__ featT, const int* __restrict__ cnt, const int* __restrict__ start,
    const int* __restrict__ perm, int c, int n, int r3, float* __restrict__ out) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (v >= r3) return;
  const size_t vi = (size_t)b * r3 + v;
  const int m = cnt[vi];
  if (m > kRankScan) return;  // vox_seg_gather_kernel
  float* O = out + (size_t)b * c * r3 + v;
  const int* P = perm + (size_t)b * n + (m > 0 ? start[vi] : 0);
  const float* FT = featT + (size_t)b * n * c;
  const float inv = m > 0 ? pcr_inv_count(m) : 0.0f;
  constexpr int kHold = 4;  // the first points' rows, read once for every chunk
  const float* rows[kHold];
#pragma unroll
  for (int s = 0; s < kHold; s++) rows[s] = s < m ? FT + (size_t)P[s] * c : FT;
  const bool vec = (c & 3) == 0;
  // every lane runs the same chunk loop and stores (empty voxels add nothing
  // and store zeros), so the stores stay whole-wave and coalesced
  for (int c0 = 0; c0 < c; c0 += CH) {
    float acc[CH];
#pragma unroll
    for (int q = 0; q < CH; q++) acc[q] = 0.0f;
    if (vec && c0 + CH <= c) {
#pragma unroll
      for (int s = 0; s < kHold; s++) {
        if (s < m) {
#pragma unroll
          for (int q = 0; q < CH; q += 4) {
            const float4 x = *reinterpret_cast<const float4*>(rows[s] + c0 + q);
            acc[q] += x.x * inv;
            acc[q + 1] += x.y * inv;
            acc[q + 2] += x.z * inv;
            acc[q + 3] += x.w * inv;
          }
        }
      }
      for (int s = kHold; s < m; s++) {
        const float* row = FT + (size_t)P[s] * c + c0;
#pragma unroll
        for (int q = 0; q < CH; q += 4) {
          const float4 x = *reinterpret_cast<const float4*>(row + q);
          acc[q] += x.x * inv;
          acc[q + 1] += x.y * inv;
          acc[q + 2] += x.z * inv;
          acc[q + 3] += x.w * inv;
        }
      }
    } else {
      for (int s = 0; s < m; s++) {
        const float* row = FT + (size_t)P[s] * c + c0;
#pragma unroll
        for (int q = 0; q < CH; q++)
          if (c0 + q < c) acc[q] += row[q] * inv;
      }
    }
#pragma unroll
    for (int q = 0; q < CH; q++)
      // nontemporal: the 537 MB grid at c5 is written once (c5 step -2%)
      if (c0 + q < c) __builtin_nontemporal_store(acc[q], &O[(size_t)(c0 + q) * r3]);
  }
}

template <int MODE>
static pcr_status run_voxelize_big(const float* features, const float* coords_f,
                                   const int* coords_i, int b, int c, int n, int r, float* out,
                                   int* ind, int* cnt, void* workspace, size_t ws_bytes,
                                   hipStream_t stream, const char* name) {
  const int r3 = r * r * r;
  PCR_REQUIRE(cnt != nullptr && ind != nullptr, "%s: ind and cnt required", name);
  PCR_REQUIRE((int64_t)b * n < (1ll << 31) && (int64_t)b * r3 < (1ll << 31),
              "%s: batch too large for the sorted path", name);
  BigVoxWs ws;
  // with room for the point-major feature copy the coalesced gather runs,
  // else the direct one (same results)
  size_t need = big_ws_layout(b, n, r, &ws, workspace, c);
  if (workspace == nullptr || ws_bytes < need) need = big_ws_layout(b, n, r, &ws, workspace, 0);
  PCR_REQUIRE(workspace != nullptr && ws_bytes >= need, "%s: workspace too small (%zu < %zu)",
              name, ws_bytes, need);
  if (hipMemsetAsync(cnt, 0, (size_t)b * r3 * sizeof(int), stream) != hipSuccess ||
      hipMemsetAsync(ws.big, 0, sizeof(int), stream) != hipSuccess) {
    set_error("%s: memset failed", name);
    return PCR_ERR_LAUNCH;
  }
  const dim3 pts(ceil_div(n, 256), b);
  hipLaunchKernelGGL(vox_key_big_kernel<MODE>, pts, dim3(256), 0, stream, coords_f, coords_i, n,
                     r, ind, cnt, ws.slot);
  if (c > 0 && out) {
    const dim3 tiles(ws.ntile, b);
    hipLaunchKernelGGL(vox_scan_tiles_kernel, tiles, dim3(kBigScanThreads), 0, stream, cnt, r3,
                       ws.ntile, ws.tsum);
    hipLaunchKernelGGL(vox_scan_apply_kernel, tiles, dim3(kBigScanThreads), 0, stream, cnt, r3,
                       ws.ntile, ws.tsum, ws.start);
    hipLaunchKernelGGL(vox_place_big_kernel, pts, dim3(256), 0, stream, ind, ws.slot, n, r3,
                       ws.start, ws.perm_u);
    hipLaunchKernelGGL(vox_rank_big_kernel, pts, dim3(256), 0, stream, ind, ws.slot, n, r3, cnt,
                       ws.start, ws.perm_u, ws.perm, ws.big);
    const int kbits = n > 1 ? 32 - __builtin_clz((unsigned)(n - 1)) : 1;
    hipLaunchKernelGGL(vox_seg_sort_kernel, dim3(64), dim3(kSegSortThreads), 0, stream, ws.big,
                       cnt, ws.start, n, r3, kbits, ws.perm_u, ws.perm);
    if (ws.featT) {
      hipLaunchKernelGGL(feat_transpose_kernel, dim3(ceil_div(n, 64), ceil_div(c, 64), b),
                         dim3(256), 0, stream, features, c, n, ws.featT);
      hipLaunchKernelGGL(vox_gather_big_t_kernel<32>, dim3(ceil_div(r3, 256), b), dim3(256), 0,
                         stream, ws.featT, cnt, ws.start, ws.perm, c, n, r3, out);
      hipLaunchKernelGGL(vox_seg_gather_kernel<true>, dim3(64), dim3(256), 0, stream, ws.big,
                         ws.featT, cnt, ws.start, ws.perm, c, n, r3, out);
    } else {
      hipLaunchKernelGGL(vox_gather_big_kernel, dim3(ceil_div(r3, 256), b), dim3(256), 0, stream,
                         features, cnt, ws.start, ws.perm, c, n, r3, out);
      hipLaunchKernelGGL(vox_seg_gather_kernel<false>, dim3(64), dim3(256), 0, stream, ws.big,
                         features, cnt, ws.start, ws.perm, c, n, r3, out);
    }
  }
  return launch_status(name);
}

// ------------------------------------------------------------- launchers
static int pick_groups(int c, int n, int max_g, int* G_out) {
  // LDS per grid WG ~ (2*G + 1) * n * 4 + bitmap: at most max_g channels
  int G = kMaxG;
  while (G > 1 && ((size_t)(2 * G + 1) * n * 4 + 8192) > 65536) G >>= 1;
  if (G > max_g) G = max_g;
  *G_out = G;
  return ceil_div(c, G);
}

static size_t grid_smem_bytes(int G, int n, int nw) {
  return ((size_t)G * n + (size_t)G * (n + 1) + (n + 1) + 2 * (size_t)nw) * 4;
}

// Launch helpers.  `what`: 1 = prep only, 2 = grid only, 3 = both.
template <int MODE>
static pcr_status run_voxelize(const float* features, const float* coords_f, const int* coords_i,
                               int b, int c, int n, int r, float* out, int* ind, int* cnt,
                               void* workspace, size_t ws_bytes, hipStream_t stream,
                               float* norm_out, float* devox, int* dinds, float* dwgts,
                               float* desc, const char* name, int what = 3) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r >= 1, "%s: invalid sizes b=%d c=%d n=%d r=%d", name,
              b, c, n, r);
  PCR_REQUIRE((int64_t)r * r * r <= (1 << 24), "%s: resolution %d too large", name, r);
  if (b == 0) return PCR_OK;
  if (n > kMaxSortN && MODE != kSphNormalize && what == 3 && devox == nullptr)
    return run_voxelize_big<MODE>(features, coords_f, coords_i, b, c, n, r, out, ind, cnt,
                                  workspace, ws_bytes, stream, name);
  PCR_REQUIRE(n >= 1 && n <= kMaxSortN,
              "%s: n=%d points per cloud unsupported on this path (1..%d)", name, n, kMaxSortN);
  const int r3 = r * r * r;
  VoxWs ws;
  size_t need = vox_ws_layout(b, n, r, &ws, workspace);
  PCR_REQUIRE(workspace != nullptr && ws_bytes >= need, "%s: workspace too small (%zu < %zu)",
              name, ws_bytes, need);
  PCR_PRIO_INIT();
  if (what & 1) {
    // clouds of <= 1024 points: a 256- or 512-thread workgroup rather than
    // 1024, so a prep workgroup fits on a CU beside the other queues'
    // kernels instead of waiting for whole CUs to drain.  257..1024 points:
    // 512 threads (two points each): under the runner's schedule 6 the prep
    // kernel heads the critical voxel chain, c2 379-385k -> 385-394k
    // clouds/s against 256 threads (3 interleaved rounds,
    // profiles/r04_ab_prep.log); 1024 threads measured between the two
    const bool small = n <= kSmallPrepN;
    const int nt = small ? kSmallPrepThreads : kPrepThreads;
    const int npad = next_pow2(n < nt ? nt : n);
    size_t prep_smem = (size_t)npad * 8 + (size_t)ws.W * 8 + (size_t)n * 8;
    PCR_REQUIRE(prep_smem <= 150 * 1024, "%s: prep LDS %zu too large", name, prep_smem);
    if (small && n > 256) {
      const int npad5 = next_pow2(n < 512 ? 512 : n);
      const size_t sm5 = (size_t)npad5 * 8 + (size_t)ws.W * 8 + (size_t)n * 8;
      allow_big_lds(vox_prep_kernel<MODE, 512>, sm5);
      hipLaunchKernelGGL((vox_prep_kernel<MODE, 512>), dim3(b), dim3(512), sm5, stream, coords_f,
                         coords_i, n, r, npad5, norm_out, ind, ws, dinds, dwgts, 1);
    } else if (small) {
      allow_big_lds(vox_prep_kernel<MODE, kSmallPrepThreads>, prep_smem);
      hipLaunchKernelGGL((vox_prep_kernel<MODE, kSmallPrepThreads>), dim3(b),
                         dim3(kSmallPrepThreads), prep_smem, stream, coords_f, coords_i, n, r,
                         npad, norm_out, ind, ws, dinds, dwgts, 1);
    } else {
      const int npad1 = next_pow2(n < kPrepThreads ? kPrepThreads : n);
      const size_t sm1 = (size_t)npad1 * 8 + (size_t)ws.W * 8 + (size_t)n * 8;
      allow_big_lds(vox_prep_kernel<MODE, kPrepThreads>, sm1);
      hipLaunchKernelGGL((vox_prep_kernel<MODE, kPrepThreads>), dim3(b), dim3(kPrepThreads),
                         sm1, stream, coords_f, coords_i, n, r, npad1, norm_out, ind, ws,
                         dinds, dwgts, 1);
    }
  }
  const bool do_grid = (what & 2) != 0;
  const bool do_dev = (what & 4) != 0 && devox != nullptr;
  // one tile covers the whole grid when its bitmap fits comfortably
  const int tile = r3 <= 65536 ? ((r3 + 31) / 32) * 32 : 32768;
  const int ntiles = ceil_div(r3, tile);
  const int nw = (tile + 31) / 32 + 1;
  if (do_dev) {
    PCR_REQUIRE(ntiles == 1, "%s: fused devoxelisation needs r^3 <= 65536", name);
    PCR_REQUIRE(c > 0, "%s: fused devoxelisation needs c > 0", name);
  }
  if (do_grid && do_dev) {
    // streaming + devox from the same LDS means: two channels per workgroup
    // as in the streaming-only part; the devox tail gathers by prep's
    // corner -> segment map
    int G = 1;
    const int ngrp = pick_groups(c, n, 2, &G);
    const size_t smem = grid_smem_bytes(G, n, nw);
    PCR_REQUIRE(smem <= 150 * 1024, "%s: grid LDS %zu too large", name, smem);
    allow_big_lds(vox_grid_kernel<3, kGridThreads, 2>, smem);
    hipLaunchKernelGGL((vox_grid_kernel<3, kGridThreads, 2>), dim3(ngrp * b),
                       dim3(kGridThreads), smem, stream, features, c, n, r3, G, tile, ws, out, cnt,
                       dinds, dwgts, devox, desc, 1, ngrp, ngrp * b);
  } else if (do_dev) {
    int G = 1;
    const int ngrp = pick_groups(c, n, 4, &G);
    const size_t smem = grid_smem_bytes(G, n, nw);
    PCR_REQUIRE(smem <= 150 * 1024, "%s: grid LDS %zu too large", name, smem);
    allow_big_lds(vox_grid_kernel<2, kDevoxThreads, 4>, smem);
    hipLaunchKernelGGL((vox_grid_kernel<2, kDevoxThreads, 4>), dim3(ngrp * b),
                       dim3(kDevoxThreads), smem, stream, features, c, n, r3, G, tile, ws, nullptr,
                       nullptr, dinds, dwgts, devox, desc, 1, ngrp, ngrp * b);
  } else if (do_grid && (c > 0 || cnt)) {
    // streaming part: two channels per workgroup keep its LDS small (~29 KB
    // at n = 1024), so its workgroups fit beside the KNN selection's
    int G = 1;
    const int ngrp = c > 0 ? pick_groups(c, n, 2, &G) : 1;
    const size_t smem = grid_smem_bytes(G, n, nw);
    PCR_REQUIRE(smem <= 150 * 1024, "%s: grid LDS %zu too large", name, smem);
    allow_big_lds(vox_grid_kernel<1, kGridThreads, 2>, smem);
    hipLaunchKernelGGL((vox_grid_kernel<1, kGridThreads, 2>),
                       dim3(ntiles * ngrp * b), dim3(kGridThreads), smem, stream,
                       features, c, n, r3, G, tile, ws, out, cnt, nullptr, nullptr, nullptr,
                       nullptr, ntiles, ngrp, ntiles * ngrp * b);
  }
  return launch_status(name);
}

}  // namespace pcr

using namespace pcr;

extern "C" size_t pcr_voxelize_workspace_size(int b, int n, int r) {
  if (b <= 0 || n <= 0 || r <= 0) return 256;
  if (n > kMaxSortN) return big_ws_layout(b, n, r, nullptr, nullptr);
  return vox_ws_layout(b, n, r, nullptr, nullptr);
}

extern "C" size_t pcr_voxelize_workspace_size_c(int b, int c, int n, int r) {
  if (b <= 0 || n <= 0 || r <= 0) return 256;
  if (n > kMaxSortN) return big_ws_layout(b, n, r, nullptr, nullptr, c > 0 ? c : 0);
  return vox_ws_layout(b, n, r, nullptr, nullptr);
}

extern "C" pcr_status pcr_spherical_avg_voxelize_forward(const float* features, const float* coords,
                                                         int b, int c, int n, int r, float* out,
                                                         int* ind, int* cnt, void* workspace,
                                                         size_t workspace_bytes, void* stream) {
  return run_voxelize<kSphCoords>(features, coords, nullptr, b, c, n, r, out, ind, cnt, workspace,
                                  workspace_bytes, as_stream(stream), nullptr, nullptr, nullptr,
                                  nullptr, nullptr, "spherical_avg_voxelize_forward");
}

extern "C" pcr_status pcr_avg_voxelize_forward(const float* features, const int* coords, int b,
                                               int c, int n, int r, float* out, int* ind, int* cnt,
                                               void* workspace, size_t workspace_bytes,
                                               void* stream) {
  return run_voxelize<kCube>(features, nullptr, coords, b, c, n, r, out, ind, cnt, workspace,
                             workspace_bytes, as_stream(stream), nullptr, nullptr, nullptr,
                             nullptr, nullptr, "avg_voxelize_forward");
}

extern "C" pcr_status pcr_avg_voxelize_backward(const float* grad_y, const int* ind,
                                                const int* cnt, int b, int c, int n, int r3,
                                                float* grad_x, void* stream) {
  PCR_REQUIRE(b >= 0 && c >= 0 && n >= 0 && r3 >= 1, "avg_voxelize_backward: invalid sizes");
  if (b == 0 || c == 0 || n == 0) return PCR_OK;
  if (n <= kGradSortMaxN && (r3 + 31) / 32 <= kGradSortMaxRows) {
    hipLaunchKernelGGL(avg_vox_grad_sorted_kernel, dim3(ceil_div(c, kGradSortCG), b),
                       dim3(kGradSortThreads), 0, as_stream(stream), grad_y, ind, cnt, c, n, r3,
                       grad_x);
    return launch_status("avg_voxelize_backward");
  }
  hipLaunchKernelGGL(avg_vox_grad_kernel, dim3(ceil_div(n, 256), ceil_div(c, kGradCG), b),
                     dim3(256), 0, as_stream(stream), grad_y, ind, cnt, c, n, r3, grad_x);
  return launch_status("avg_voxelize_backward");
}

extern "C" pcr_status pcr_spherical_normalize(const float* coords, int b, int n,
                                              float* norm_coords, void* stream) {
  PCR_REQUIRE(b >= 0 && n >= 1, "spherical_normalize: invalid sizes b=%d n=%d", b, n);
  if (b == 0) return PCR_OK;
  if (n > kMaxSortN) {
    hipLaunchKernelGGL(sph_normalize_big_kernel, dim3(b), dim3(kPrepThreads), 0,
                       as_stream(stream), coords, n, norm_coords);
    return launch_status("spherical_normalize");
  }
  const int E = next_pow2(n < kPrepThreads ? kPrepThreads : n) / kPrepThreads;
  hipLaunchKernelGGL(sph_normalize_kernel, dim3(b), dim3(kPrepThreads), 0, as_stream(stream),
                     coords, n, E, norm_coords);
  return launch_status("spherical_normalize");
}

extern "C" size_t pcr_extractor_workspace_size(int b, int n, int c, int r) {
  if (b <= 0 || n <= 0 || r <= 0) return 256;
  return vox_ws_layout(b, n, r, nullptr, nullptr, c > 0 ? c : 0);
}

// The extractor's voxel stage as prep -> means/devox -> stream (the split
// that lets the dense grid stream beside the KNN selection):
static pcr_status extractor_ws(int b, int c, int n, int r, void* workspace, size_t ws_bytes,
                               VoxWs* ws, const char* name) {
  PCR_REQUIRE(b >= 0 && c >= 1 && n >= 1 && n <= kMaxSortN && r >= 1,
              "%s: invalid sizes b=%d c=%d n=%d r=%d", name, b, c, n, r);
  const int64_t r3 = (int64_t)r * r * r;
  PCR_REQUIRE(r3 <= 65536 && r3 % 4 == 0, "%s: resolution %d unsupported (r^3 <= 65536, r^3 %% 4 == 0)",
              name, r);
  const size_t need = vox_ws_layout(b, n, r, ws, workspace, c);
  PCR_REQUIRE(workspace != nullptr && ws_bytes >= need, "%s: workspace too small (%zu < %zu)",
              name, ws_bytes, need);
  return PCR_OK;
}

extern "C" pcr_status pcr_extractor_voxel_means_devox(const float* features, int b, int c, int n,
                                                      int r, float* devox, const int* dinds,
                                                      const float* dwgts, float* desc,
                                                      void* workspace, size_t workspace_bytes,
                                                      void* stream) {
  const char* name = "extractor_voxel_means_devox";
  PCR_PRIO_INIT();
  VoxWs ws;
  pcr_status rc = extractor_ws(b, c, n, r, workspace, workspace_bytes, &ws, name);
  if (rc != PCR_OK) return rc;
  PCR_REQUIRE(devox != nullptr && dinds != nullptr && dwgts != nullptr,
              "%s: devox, dinds, dwgts required", name);
  if (b == 0) return PCR_OK;
  const int r3 = r * r * r;
  const int tile = ((r3 + 31) / 32) * 32;
  const int nw = tile / 32 + 1;
  if (n <= kMeansMaxN) {
    // 2 channels per workgroup (~24 KB of LDS, so it fits beside the KNN
    // selection's workgroups); clouds of more than 1024 points (c3: 2048):
    // 512 threads, the same four points per thread (4 or 8 channels per
    // workgroup measured +1% / -2% in the c2 step)
    const int nt = n > kMeansPB * kMeansNT ? 2 * kMeansNT : kMeansNT;
    const int ngrp = ceil_div(c, 2);
    const size_t smem = ((size_t)2 * n + (size_t)2 * (n + 1) + n + (n + 1)) * 4;
    if (nt == kMeansNT) {
      allow_big_lds(vox_means_kernel<2, kMeansNT>, smem);
      hipLaunchKernelGGL((vox_means_kernel<2, kMeansNT>), dim3(ngrp * b), dim3(kMeansNT), smem,
                         as_stream(stream), features, c, n, ws, dwgts, devox, desc, ngrp);
    } else {
      allow_big_lds(vox_means_kernel<2, 2 * kMeansNT>, smem);
      hipLaunchKernelGGL((vox_means_kernel<2, 2 * kMeansNT>), dim3(ngrp * b), dim3(2 * kMeansNT),
                         smem, as_stream(stream), features, c, n, ws, dwgts, devox, desc, ngrp);
    }
    return launch_status(name);
  }
  // larger clouds: the grid kernel's devox part (means formed per workgroup)
  int G = 1;
  const int ngrp = pick_groups(c, n, 2, &G);
  const size_t smem = grid_smem_bytes(G, n, nw);
  PCR_REQUIRE(smem <= 150 * 1024, "%s: LDS %zu too large", name, smem);
  allow_big_lds(vox_grid_kernel<2, 256, 2>, smem);
  hipLaunchKernelGGL((vox_grid_kernel<2, 256, 2>), dim3(ngrp * b), dim3(256), smem,
                     as_stream(stream), features, c, n, r3, G, tile, ws, nullptr, nullptr, dinds,
                     dwgts, devox, desc, 1, ngrp, ngrp * b);
  return launch_status(name);
}

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

extern "C" pcr_status pcr_extractor_voxel_stream(int b, int c, int n, int r, int* cnt,
                                                 float* grid, void* workspace,
                                                 size_t workspace_bytes, void* stream) {
  const char* name = "extractor_voxel_stream";
  PCR_PRIO_INIT();
  VoxWs ws;
  pcr_status rc = extractor_ws(b, c, n, r, workspace, workspace_bytes, &ws, name);
  if (rc != PCR_OK) return rc;
  PCR_REQUIRE(grid != nullptr, "%s: grid required", name);
  if (b == 0) return PCR_OK;
  const int r3 = r * r * r;
  PCR_REQUIRE(n <= kStreamMaxN && r3 <= 32 * kStreamMaxW && r3 % 128 == 0,
              "%s: n=%d r=%d unsupported (n <= %d, r^3 <= %d, r^3 %% 128 == 0)", name, n, r,
              kStreamMaxN, 32 * kStreamMaxW);
  // two channels per item and three means buffers: 36 KB, so the grid
  // kernel fits on a CU beside two selection workgroups (four channels per
  // item measured ~3% slower in the step despite half the index work per
  // store); clouds of more than 1024 points (c3): 17 pieces per item
  const bool wide = n > 1024;
  constexpr int G = kStreamG;
  const int NGP = wide ? 17 : kStreamNG;  // 1 KB pieces holding G rows of ms floats
  PCR_REQUIRE(G * ws.ms * 4 <= NGP * 1024, "%s: means rows too long", name);
  const int ngrp = ceil_div(c, G);
  // a few workgroups per cloud (about one per CU in all), each a contiguous
  // range of channel-group items of that cloud
  int wpc = device_cus() / (b > 0 ? b : 1);
  if (wpc < 1) wpc = 1;
  if (wpc > ngrp) wpc = ngrp;
  const int per = ceil_div(ngrp, wpc);
  PCR_REQUIRE(ws.W % 64 == 0, "%s: r^3 %% 2048 != 0 unsupported", name);
  const size_t smem = stream_smem_bytes(NGP, ws.W, ws.ms);
#define PCR_LAUNCH_STREAM(NGV)                                                                 \
  do {                                                                                        \
    allow_big_lds(vox_stream_kernel<4, kStreamNB, 2, 16, G, NGV>, smem);                      \
    hipLaunchKernelGGL((vox_stream_kernel<4, kStreamNB, 2, 16, G, NGV>), dim3(b * wpc),       \
                       dim3(5 * 64), smem, as_stream(stream), c, n, r3, ws, grid, cnt, ngrp,   \
                       wpc, per, nullptr, nullptr, nullptr);                                  \
  } while (0)
  if (wide) PCR_LAUNCH_STREAM(17);
  else PCR_LAUNCH_STREAM(kStreamNG);
#undef PCR_LAUNCH_STREAM
  return launch_status(name);
}

// The voxel stage's back half with the devox inside the grid stream
// (vox_stream_kernel<..., DV = true>): the means launch writes only the
// compact means rows (vox_means_kernel<2, 256, false>), then the grid stream
// writes grid + cnt and, from the same means in LDS, devox [b,c,n] and the
// descriptor [b,c].  Same outputs, bits and order of operations as
// pcr_extractor_voxel_means_devox + pcr_extractor_voxel_stream; clouds of at
// most 1024 points (pcr_extractor_stream_devox_ok).
extern "C" int pcr_extractor_stream_devox_ok(int n, int c, int r) {
  const int r3 = r * r * r;
  return n >= 1 && n <= kStreamDvMaxN && c >= 1 && r3 <= 32 * kStreamMaxW && r3 % 2048 == 0;
}

extern "C" pcr_status pcr_extractor_voxel_means(const float* features, int b, int c, int n, int r,
                                                void* workspace, size_t workspace_bytes,
                                                void* stream) {
  const char* name = "extractor_voxel_means";
  VoxWs ws;
  pcr_status rc = extractor_ws(b, c, n, r, workspace, workspace_bytes, &ws, name);
  if (rc != PCR_OK) return rc;
  PCR_REQUIRE(features != nullptr && n <= kMeansMaxN, "%s: features required, n <= %d", name,
              kMeansMaxN);
  if (b == 0) return PCR_OK;
  const int ngrp = ceil_div(c, 2);
  const size_t smem = ((size_t)2 * n + (size_t)2 * (n + 1) + n + (n + 1)) * 4;
  // clouds of more than 1024 points: 512 threads, the same four points per thread
  if (n > kMeansPB * kMeansNT) {
    allow_big_lds(vox_means_kernel<2, 2 * kMeansNT, false>, smem);
    hipLaunchKernelGGL((vox_means_kernel<2, 2 * kMeansNT, false>), dim3(ngrp * b),
                       dim3(2 * kMeansNT), smem, as_stream(stream), features, c, n, ws, nullptr,
                       nullptr, nullptr, ngrp);
  } else {
    allow_big_lds(vox_means_kernel<2, kMeansNT, false>, smem);
    hipLaunchKernelGGL((vox_means_kernel<2, kMeansNT, false>), dim3(ngrp * b), dim3(kMeansNT),
                       smem, as_stream(stream), features, c, n, ws, nullptr, nullptr, nullptr,
                       ngrp);
  }
  return launch_status(name);
}

extern "C" pcr_status pcr_extractor_voxel_stream_devox(int b, int c, int n, int r, int* cnt,
                                                       float* grid, float* devox,
                                                       const float* dwgts, float* desc,
                                                       void* workspace, size_t workspace_bytes,
                                                       void* stream) {
  const char* name = "extractor_voxel_stream_devox";
  VoxWs ws;
  pcr_status rc = extractor_ws(b, c, n, r, workspace, workspace_bytes, &ws, name);
  if (rc != PCR_OK) return rc;
  PCR_REQUIRE(grid != nullptr && devox != nullptr && dwgts != nullptr,
              "%s: grid, devox and dwgts required", name);
  PCR_REQUIRE(pcr_extractor_stream_devox_ok(n, c, r), "%s: n=%d c=%d r=%d unsupported", name, n,
              c, r);
  if (b == 0) return PCR_OK;
  const int r3 = r * r * r;
  constexpr int G = kStreamG;
  const int NGP = kStreamNG;
  PCR_REQUIRE(G * ws.ms * 4 <= NGP * 1024, "%s: means rows too long", name);
  const int ngrp = ceil_div(c, G);
  int wpc = device_cus() / b;
  if (wpc < 1) wpc = 1;
  if (wpc > ngrp) wpc = ngrp;
  const int per = ceil_div(ngrp, wpc);
  const size_t smem = stream_smem_bytes(NGP, ws.W, ws.ms);
  allow_big_lds(vox_stream_kernel<4, kStreamNB, 2, 16, G, kStreamNG, kStreamDvMaxN>, smem);
  hipLaunchKernelGGL((vox_stream_kernel<4, kStreamNB, 2, 16, G, kStreamNG, kStreamDvMaxN>),
                     dim3(b * wpc), dim3(5 * 64), smem, as_stream(stream), c, n, r3, ws, grid, cnt,
                     ngrp, wpc, per, dwgts, devox, desc);
  return launch_status(name);
}

extern "C" pcr_status pcr_extractor_voxel_prep(const float* xyz, int b, int n, int r,
                                               float* norm_coords, int* ind, int* dinds,
                                               float* dwgts, void* workspace,
                                               size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(ind != nullptr && dinds != nullptr && dwgts != nullptr,
              "extractor_voxel_prep: ind, dinds, dwgts required");
  return run_voxelize<kSphNormalize>(nullptr, xyz, nullptr, b, 0, n, r, nullptr, ind, nullptr,
                                     workspace, workspace_bytes, as_stream(stream), norm_coords,
                                     nullptr, dinds, dwgts, nullptr, "extractor_voxel_prep", 1);
}

extern "C" pcr_status pcr_extractor_voxel_grid(const float* features, int b, int c, int n, int r,
                                               int* cnt, float* grid, void* workspace,
                                               size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(grid != nullptr, "extractor_voxel_grid: grid required");
  return run_voxelize<kSphNormalize>(features, nullptr, nullptr, b, c, n, r, grid, nullptr, cnt,
                                     workspace, workspace_bytes, as_stream(stream), nullptr,
                                     nullptr, nullptr, nullptr, nullptr, "extractor_voxel_grid", 2);
}

extern "C" pcr_status pcr_extractor_voxel_devox(const float* features, int b, int c, int n, int r,
                                                float* devox, const int* dinds, const float* dwgts,
                                                float* desc, void* workspace,
                                                size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(devox != nullptr && dinds != nullptr && dwgts != nullptr,
              "extractor_voxel_devox: devox, dinds, dwgts required");
  return run_voxelize<kSphNormalize>(features, nullptr, nullptr, b, c, n, r, nullptr, nullptr,
                                     nullptr, workspace, workspace_bytes, as_stream(stream), nullptr,
                                     devox, const_cast<int*>(dinds), const_cast<float*>(dwgts),
                                     desc, "extractor_voxel_devox", 4);
}

extern "C" pcr_status pcr_extractor_voxel_grid_devox(const float* features, int b, int c, int n,
                                                     int r, int* cnt, float* grid, float* devox,
                                                     const int* dinds, const float* dwgts,
                                                     float* desc, void* workspace,
                                                     size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(grid != nullptr && devox != nullptr && dinds != nullptr && dwgts != nullptr,
              "extractor_voxel_grid_devox: grid, devox, dinds, dwgts required");
  return run_voxelize<kSphNormalize>(features, nullptr, nullptr, b, c, n, r, grid, nullptr, cnt,
                                     workspace, workspace_bytes, as_stream(stream), nullptr,
                                     devox, const_cast<int*>(dinds), const_cast<float*>(dwgts),
                                     desc, "extractor_voxel_grid_devox", 6);
}

extern "C" pcr_status pcr_extractor_voxel_stage(const float* xyz, const float* features, int b,
                                                int c, int n, int r, float* norm_coords, int* ind,
                                                int* cnt, float* grid, float* devox, int* dinds,
                                                float* dwgts, float* desc, void* workspace,
                                                size_t workspace_bytes, void* stream) {
  PCR_REQUIRE(grid != nullptr && ind != nullptr, "extractor_voxel_stage: grid and ind required");
  PCR_REQUIRE(devox == nullptr || (dinds != nullptr && dwgts != nullptr),
              "extractor_voxel_stage: devox needs dinds/dwgts buffers");
  PCR_REQUIRE(desc == nullptr || devox != nullptr, "extractor_voxel_stage: desc needs devox");
  return run_voxelize<kSphNormalize>(features, xyz, nullptr, b, c, n, r, grid, ind, cnt, workspace,
                                     workspace_bytes, as_stream(stream), norm_coords, devox,
                                     dinds, dwgts, desc, "extractor_voxel_stage", 7);
}

#ifdef PCR_DIAG
PCR_DIAG_READER(pcr_diag_read_vox)
#endif
