/*
 * pcr_amd.h -- C ABI of libpcr_amd.so, the MI355X (gfx950) implementation of
 * the rotation-invariant-feature hot path of
 * Gilgamesh666666/Point-cloud-registration-based-on-rotation-invariant-feature.
 *
 * Each entry point replaces one function of the reference's pybind11 module
 * `_multi_shape_pvcnn_backend` (PVCNN/modules/functional/src/bindings.cpp) or
 * one PyTorch block of the reference model; the citation above every
 * declaration names the interface it replaces (paths relative to the
 * reference's PVCNN/ directory).
 *
 * Conventions
 *  - Plain device pointers (HIP device memory), sizes as int, layouts exactly
 *    as the reference's tensors (channel-major [B, C, N] fp32, int32 indices).
 *  - The caller owns every buffer.  Outputs are FULLY written by the library,
 *    including the slots the reference leaves at their torch::zeros /
 *    ones*10000 fill, so callers may pass uninitialised (torch.empty) memory.
 *  - `stream` is a hipStream_t (NULL = legacy default stream).  Work is only
 *    enqueued; nothing synchronises, allocates or frees, so every call is
 *    hipGraph-capturable.  Calls needing scratch take a caller-provided
 *    workspace whose size comes from the matching *_workspace_size().
 *  - Return value: PCR_OK or a negative pcr_status; pcr_last_error() holds a
 *    message (thread-local).  The reference instead exit(-1)s on a launch
 *    failure (src/cuda_utils.cuh:28-37).
 */
#ifndef PCR_AMD_H
#define PCR_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int pcr_status;
#define PCR_OK 0
#define PCR_ERR_INVALID (-1)
#define PCR_ERR_LAUNCH (-2)
#define PCR_ERR_UNSUPPORTED (-3)

/* Last error message of the calling thread ("" when none). */
const char *pcr_last_error(void);
/* Library version string. */
const char *pcr_version(void);
/* A HIP stream restricted to the CUs set in mask (nwords 32-bit words, bit
 * i = CU i of the runtime's numbering; hipExtStreamCreateWithCUMask), and its
 * release.  No reference counterpart: a scheduling tool for the runner's
 * queues. */
pcr_status pcr_stream_create_cu_mask(const unsigned *mask, int nwords, void **stream);
pcr_status pcr_stream_destroy(void *stream);

/* ---------------------------------------------------------------- KNN ----
 * knn_forward_cuda (modules/functional/src/knn/knn.cpp:6-25, kernel
 * knn/knn.cu:5-49, both directions): xyz1 [b,c,n], xyz2 [b,c,m] ->
 * dist1 [b,k,n], idx1 [b,k,n] (into xyz2), dist2 [b,k,m], idx2 [b,k,m].
 * Squared L2, ascending, ties by lower index, unfilled slots (10000, 0). */
pcr_status pcr_knn_forward(const float *xyz1, const float *xyz2, int b, int c, int n, int m,
                           int k, float *dist1, float *dist2, int *idx1, int *idx2,
                           void *workspace, size_t workspace_bytes, void *stream);
/* Scratch of the spatially pruned KNN (Morton-sorted copies + block boxes of
 * both point sets).  With workspace == NULL (or c != 3, or more than 4096
 * points per cloud) a brute-force kernel is used instead, same results. */
size_t pcr_knn_workspace_size(int b, int n, int m);

/* knn_backward_cuda (knn/knn.cpp:27-52, kernel knn/knn.cu:52-78, :88-98).
 * gradxyz1 [b,c,n], gradxyz2 [b,c,m]; both directions accumulate into both. */
pcr_status pcr_knn_backward(const float *xyz1, const float *xyz2, const float *graddist1,
                            const float *graddist2, const int *idx1, const int *idx2, int b,
                            int c, int n, int m, int k, float *gradxyz1, float *gradxyz2,
                            void *stream);
/* The same without atomics (bit-repeatable): each direction's (query, slot)
 * pairs counting-sorted by neighbour in `workspace`
 * (pcr_knn_backward_workspace_size bytes), then one gather per point of its
 * own terms and of the pairs naming it.  Clouds of more than 16384 points
 * take pcr_knn_backward. */
size_t pcr_knn_backward_workspace_size(int b, int n, int m, int k);
pcr_status pcr_knn_backward_ws(const float *xyz1, const float *xyz2, const float *graddist1,
                               const float *graddist2, const int *idx1, const int *idx2, int b,
                               int c, int n, int m, int k, float *gradxyz1, float *gradxyz2,
                               void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------- PPF ----
 * spherical_ppf_forward (modules/functional/src/spherical_ppf/ppf.cpp:17-36,
 * kernel ppf.cu:19-92).  Argument order of the BACKEND (points first); the
 * Python ppf() wrapper swaps (modules/functional/ppf.py:20).
 * coords/center/normals/center_normal [b,3,n] -> feat [b,4,n]. */
pcr_status pcr_spherical_ppf_forward(const float *coords, const float *center,
                                     const float *normals, const float *center_normal, int b,
                                     int n, float *feat, void *stream);

/* Local k-neighbour PPF of the model (models/pvcnn_classify.py:252-269:
 * BallQuery grouping of coords+normals, d = c - (p - c), three acos + |d|),
 * fused with the grouping.  points/normals [b,3,n]; centers/center_normals
 * [b,3,m]; idx either [b,m,u] (ball_query layout, idx_kmajor=0) or [b,u,m]
 * (knn layout, idx_kmajor=1).  relative=1 reproduces the model (grouped
 * coordinates are relative to the centre), relative=0 uses d = c - p.
 * out [b,4,u,m] = (nr_d, ni_d, nr_ni, |d|). */
pcr_status pcr_local_ppf_forward(const float *points, const float *normals, const float *centers,
                                 const float *center_normals, const int *idx, int b, int n,
                                 int m, int u, int idx_kmajor, int relative, float *out,
                                 void *stream);

/* Fused self-KNN + local PPF (the extractor's neighbour stage): for every
 * point of xyz [b,3,n] its k nearest points (self included, knn semantics)
 * -> idx [b,k,n], dist [b,k,n] (may be NULL) and the local PPF
 * [b,4,k,n] of (point, neighbour) with `relative` as above.  Workspace:
 * pcr_knn_workspace_size(b, n, n). */
pcr_status pcr_knn_local_ppf(const float *xyz, const float *normals, int b, int n, int k,
                             int relative, int *idx, float *dist, float *ppf, void *workspace,
                             size_t workspace_bytes, void *stream);

/* The two launches of pcr_knn_local_ppf, separately, so a pipelined caller
 * can sort step i+1 while step i selects (double-buffered workspaces):
 * prepare = Morton sort of xyz into the workspace, prepared = selection +
 * PPF from that workspace (ppf == NULL: selection only; the PPF can then
 * come from pcr_local_ppf_forward with idx_kmajor = 1, one thread per
 * output, coalesced).  Both return PCR_ERR_UNSUPPORTED (nothing
 * launched) where the sorted path does not apply (n > 4096); use
 * pcr_knn_local_ppf there. */
pcr_status pcr_knn_prepare(const float *xyz, int b, int n, void *workspace,
                           size_t workspace_bytes, void *stream);
pcr_status pcr_knn_local_ppf_prepared(const float *xyz, const float *normals, int b, int n, int k,
                                      int relative, int *idx, float *dist, float *ppf,
                                      const void *workspace, size_t workspace_bytes,
                                      void *stream);
/* Selection + local PPF of a prepared workspace in two launches whose only
 * scattered traffic is a read: the selection emits its neighbour ids in
 * sorted (Morton) query order into the workspace -- whole rows -- and the PPF
 * kernel reads them back through the sort's inverse permutation while it
 * writes knn_idx [b,k,n] (original order) and ppf [b,4,k,n].  k <= 32 and
 * n <= 2048 take that path; other shapes run pcr_knn_local_ppf_prepared +
 * pcr_local_ppf_forward.  Same outputs as those two calls. */
pcr_status pcr_knn_select_ppf(const float *xyz, const float *normals, int b, int n, int k,
                              int relative, int *idx, float *ppf, const void *workspace,
                              size_t workspace_bytes, void *stream);
/* The two launches of pcr_knn_select_ppf separately: the selection into the
 * workspace's sorted-order rows (PCR_ERR_UNSUPPORTED, nothing launched, when
 * that path does not apply), then the PPF launch that writes knn_idx and
 * ppf from them (k <= 32, n <= 2048). */
pcr_status pcr_knn_select_sorted(const float *xyz, int b, int n, int k, const void *workspace,
                                 size_t workspace_bytes, void *stream);
pcr_status pcr_knn_ppf_sorted(const float *xyz, const float *normals, int b, int n, int k,
                              int relative, int *idx, float *ppf, const void *workspace,
                              size_t workspace_bytes, void *stream);

/* ------------------------------------------------ ball query / grouping --
 * ball_query (ball_query/ball_query.cpp:6-30, kernel ball_query.cu:19-50):
 * centers [b,3,m], points [b,3,n] -> idx [b,m,u]. */
pcr_status pcr_ball_query(const float *centers, const float *points, int b, int m, int n,
                          float radius, int u, int *idx, void *stream);

/* grouping_forward (grouping/grouping.cpp:6-24, grouping.cu:18-36):
 * features [b,c,n], indices [b,m,u] -> out [b,c,m,u]. */
pcr_status pcr_grouping_forward(const float *features, const int *indices, int b, int c, int n,
                                int m, int u, float *out, void *stream);

/* grouping_backward (grouping.cpp:26-44, grouping.cu:58-85):
 * grad_y [b,c,m,u], indices [b,m,u] -> grad_x [b,c,n]. */
pcr_status pcr_grouping_backward(const float *grad_y, const int *indices, int b, int c, int n,
                                 int m, int u, float *grad_x, void *stream);

/* ------------------------------------------------------- voxelization ----
 * Scratch for the voxelizers: per-cloud sort permutation, occupied-voxel
 * segments and an occupancy bitmap with word prefix counts. */
size_t pcr_voxelize_workspace_size(int b, int n, int r);
/* The same for c feature channels.  Clouds of more than 4096 points use the
 * sorted large-cloud path; with this size it also keeps a point-major copy
 * of the features, so each voxel reads its points' channels contiguously
 * (several times faster).  The results are identical either way. */
size_t pcr_voxelize_workspace_size_c(int b, int c, int n, int r);

/* spherical_avg_voxelize_forward (spherical_voxelization/spherical_vox.cpp:17-46,
 * kernels spherical_vox.cu:19-125): features [b,c,n], normalised coords
 * [b,3,n] -> out [b,c,r^3] (voxel mean), ind [b,n] (-1 = dropped),
 * cnt [b,r^3].  Means are accumulated in ascending point order. */
pcr_status pcr_spherical_avg_voxelize_forward(const float *features, const float *coords, int b,
                                              int c, int n, int r, float *out, int *ind, int *cnt,
                                              void *workspace, size_t workspace_bytes,
                                              void *stream);

/* avg_voxelize_forward (voxelization/vox.cpp:17-46, vox.cu:18-73): cube
 * variant on int voxel coords [b,3,n]. */
pcr_status pcr_avg_voxelize_forward(const float *features, const int *coords, int b, int c,
                                    int n, int r, float *out, int *ind, int *cnt,
                                    void *workspace, size_t workspace_bytes, void *stream);

/* spherical_avg_voxelize_backward (spherical_vox.cpp:57-79, spherical_vox.cu:139-163)
 * and avg_voxelize_backward (vox.cpp:57-76, vox.cu:87-111): grad_y [b,c,r3],
 * ind [b,n], cnt [b,r3] -> grad_x [b,c,n]. */
pcr_status pcr_avg_voxelize_backward(const float *grad_y, const int *ind, const int *cnt, int b,
                                     int c, int n, int r3, float *grad_x, void *stream);

/* Spherical_Voxelization's coordinate normalisation
 * (modules/spherical_vox.py:16-20) with a fixed reduction order:
 * coords [b,3,n] -> norm_coords [b,3,n]. */
pcr_status pcr_spherical_normalize(const float *coords, int b, int n, float *norm_coords,
                                   void *stream);

/* ----------------------------------------------------- devoxelization ----
 * spherical_trilinear_devoxelize_forward
 * (interpolate/spherical_trilinear_devox.cpp:19-56, .cu:23-136): coords
 * [b,3,n], features [b,c,r^3], g_inds [b,n] -> outs [b,c,n], inds [b,8,n],
 * wgts [b,8,n].  is_training is ignored, as in the reference. */
pcr_status pcr_spherical_trilinear_devoxelize_forward(int r, int is_training, const float *coords,
                                                      const float *features, const int *g_inds,
                                                      int b, int c, int n, float *outs, int *inds,
                                                      float *wgts, void *stream);

/* trilinear_devoxelize_forward (interpolate/trilinear_devox.cpp:18-56,
 * .cu:22-106): cube variant on continuous voxel coords [b,3,n]. */
pcr_status pcr_trilinear_devoxelize_forward(int r, int is_training, const float *coords,
                                            const float *features, int b, int c, int n,
                                            float *outs, int *inds, float *wgts, void *stream);

/* spherical_trilinear_devoxelize_backward (spherical_trilinear_devox.cpp:68-92,
 * .cu:150-194; skip_neg=1: points with inds[0]==-1 are skipped) and
 * trilinear_devoxelize_backward (trilinear_devox.cpp:58-91, .cu:120-163;
 * skip_neg=0): grad_y [b,c,n] -> grad_x [b,c,r^3]. */
pcr_status pcr_devoxelize_backward(const float *grad_y, const int *inds, const float *wgts, int b,
                                   int c, int n, int r, int skip_neg, float *grad_x,
                                   void *stream);
/* The same with a workspace of pcr_devoxelize_backward_workspace_size(b, n)
 * bytes: spherical grads of clouds of <= 4096 points first sort each cloud's
 * points by corner set once (instead of every channel-group workgroup
 * sorting every 64 points), so the backward only sums runs.  Same results
 * up to the fp32 summation order of the atomics (as the reference's). */
size_t pcr_devoxelize_backward_workspace_size(int b, int n);
/* Workspace for pcr_devoxelize_backward_ws that also covers the cube
 * gather path (spherical=0, r <= 32): each cloud's 8n (point, corner) pairs
 * are counting-sorted by voxel once and every voxel sums its own segment, so
 * grad_x is written once with no atomics (trilinear_devox.cu:120-163 does one
 * global float atomic per pair and channel).  Same results up to the fp32
 * summation order within a voxel.  With only
 * pcr_devoxelize_backward_workspace_size(b, n) bytes the cube grads take
 * the LDS-atomic kernel. */
size_t pcr_devoxelize_backward_workspace_size_r(int b, int n, int r, int spherical);
pcr_status pcr_devoxelize_backward_ws(const float *grad_y, const int *inds, const float *wgts,
                                      int b, int c, int n, int r, int skip_neg, float *grad_x,
                                      void *workspace, size_t workspace_bytes, void *stream);

/* PVConv dgcnn centre term (modules/pvconv.py:68-89): related[b,c,i] =
 * features[b,c,i] - avg_grid[b,c,ind[b,i]], 0 where ind == -1. */
pcr_status pcr_dgcnn_center_gather(const float *features, const float *avg_grid, const int *ind,
                                   int b, int c, int n, int r3, float *related, void *stream);

/* ---------------------------------------------------- fused extractor ----
 * The spherical voxel stage of the sph-dg extractor forward, fused:
 * normalise coords -> spherical voxel index -> voxel mean grid (written
 * once, coalesced) -> spherical devoxelisation of that grid -> per-cloud
 * max-pooled descriptor.  Outputs (any may be NULL except grid):
 * norm_coords [b,3,n], ind [b,n], cnt [b,r^3], grid [b,c,r^3],
 * devox [b,c,n], dinds [b,8,n], dwgts [b,8,n], desc [b,c] (max over points of
 * devox).  Equivalent to pcr_spherical_normalize + ..._avg_voxelize_forward +
 * ..._trilinear_devoxelize_forward on the produced grid. */
size_t pcr_extractor_workspace_size(int b, int n, int c, int r);
pcr_status pcr_extractor_voxel_stage(const float *xyz, const float *features, int b, int c,
                                     int n, int r, float *norm_coords, int *ind, int *cnt,
                                     float *grid, float *devox, int *dinds, float *dwgts,
                                     float *desc, void *workspace, size_t workspace_bytes,
                                     void *stream);

/* The launches of pcr_extractor_voxel_stage, separately, so a caller can run
 * the grid and devox launches on two streams (they are independent once prep
 * is done) and time the grid kernel with events on its stream:
 *   prep  = normalise + voxel index + occupancy/segments + devox corners
 *   grid  = voxel means -> dense grid [b,c,r^3] + cnt, written once
 *   devox = voxel means -> spherical devoxelisation [b,c,n] + descriptor
 * The workspace carries the prep results to the other two. */
pcr_status pcr_extractor_voxel_prep(const float *xyz, int b, int n, int r, float *norm_coords,
                                    int *ind, int *dinds, float *dwgts, void *workspace,
                                    size_t workspace_bytes, void *stream);
pcr_status pcr_extractor_voxel_grid(const float *features, int b, int c, int n, int r, int *cnt,
                                    float *grid, void *workspace, size_t workspace_bytes,
                                    void *stream);
pcr_status pcr_extractor_voxel_devox(const float *features, int b, int c, int n, int r,
                                     float *devox, const int *dinds, const float *dwgts,
                                     float *desc, void *workspace, size_t workspace_bytes,
                                     void *stream);
/* devox + descriptor from the dense grid the grid launch wrote (on the same
 * stream, after it): every spherical corner lies in a fixed set of 80 voxels
 * (spherical_trilinear_devox.cu:67-105), whose values are staged in LDS per
 * channel; corners from prep's dinds / dwgts.  n <= 4096.  Same outputs as
 * pcr_extractor_voxel_devox (which re-forms the voxel means from the
 * features instead of reading the grid). */
pcr_status pcr_extractor_grid_devox(const float *grid, const int *dinds, const float *dwgts,
                                    int b, int c, int n, int r, float *devox, float *desc,
                                    void *stream);
/* grid + devox + descriptor in one launch after prep (the devox tail gathers
 * the voxel means the workgroup already holds in LDS, through prep's corner
 * -> segment map): what pcr_extractor_voxel_stage launches after prep. */
pcr_status pcr_extractor_voxel_grid_devox(const float *features, int b, int c, int n, int r,
                                          int *cnt, float *grid, float *devox, const int *dinds,
                                          const float *dwgts, float *desc, void *workspace,
                                          size_t workspace_bytes, void *stream);

/* The voxel stage split so the dense grid streams beside the KNN selection
 * (what vox_grid_kernel<3> does in one launch, in two):
 *   means_devox: the voxel means of every occupied segment (fixed ascending
 *     point order) into the workspace, spherical_trilinear_devoxelize of them
 *     (spherical_trilinear_devox.cu:23-136) and the per-cloud descriptor;
 *   stream: the dense [B, C, r^3] grid + cnt [B, r^3] of
 *     spherical_avg_voxelize_forward (spherical_vox.cu:19-125) from those
 *     means, written once, zeros included.
 * Both read the workspace pcr_extractor_voxel_prep filled; its size is
 * pcr_extractor_workspace_size(b, n, c, r).  r^3 <= 65536, r^3 % 4 == 0. */
pcr_status pcr_extractor_voxel_means_devox(const float *features, int b, int c, int n, int r,
                                           float *devox, const int *dinds, const float *dwgts,
                                           float *desc, void *workspace, size_t workspace_bytes,
                                           void *stream);
pcr_status pcr_extractor_voxel_stream(int b, int c, int n, int r, int *cnt, float *grid,
                                      void *workspace, size_t workspace_bytes, void *stream);
/* The same back half with the spherical devox moved into the grid stream:
 * pcr_extractor_voxel_means writes only the compact means rows (no devox,
 * no descriptor), then pcr_extractor_voxel_stream_devox writes grid + cnt,
 * devox [b,c,n] (from dwgts and prep's corner segments) and desc [b,c]
 * (NULL: none) -- the outputs of means_devox + stream, bit for bit, with the
 * cloud's corner data read once per grid workgroup instead of once per
 * channel pair.  pcr_extractor_stream_devox_ok(n, c, r) is nonzero where it
 * applies (n <= 1024, r^3 <= 32768). */
int pcr_extractor_stream_devox_ok(int n, int c, int r);
pcr_status pcr_extractor_voxel_means(const float *features, int b, int c, int n, int r,
                                     void *workspace, size_t workspace_bytes, void *stream);
pcr_status pcr_extractor_voxel_stream_devox(int b, int c, int n, int r, int *cnt, float *grid,
                                            float *devox, const float *dwgts, float *desc,
                                            void *workspace, size_t workspace_bytes,
                                            void *stream);

/* ------------------------------------------- mutual-NN matching (8f f1) ----
 * datasets/deepgmr_mn40.py:232-244 find_correspondence_one_pair, for p pairs:
 * f1 [p, n1, c], f2 [p, n2, c] (rows = points, channels contiguous, as the
 * numpy [n, c] arrays).  diff = |f1_i|^2 + |f2_j|^2 - 2 f1_i . f2_j;
 * corr12 [p, n1] = argmin_j, corr21 [p, n2] = argmin_i (first index on ties,
 * NaN first as np.argmin); idx1 / idx2 [p, n1] = the mutual pairs
 * (corr21[corr12[i]] == i) in ascending i, -1 after count[p] of them.
 * Channel sums are k-ordered fmaf chains (fp32 MFMA), include/pcr_math.h. */
size_t pcr_mutual_nn_workspace_size(int p, int n1, int n2);
pcr_status pcr_mutual_nn_match(const float *f1, const float *f2, int p, int n1, int n2, int c,
                               int *corr12, int *corr21, int *idx1, int *idx2, int *count,
                               void *workspace, size_t workspace_bytes, void *stream);
/* The same on channel-major per-point features -- f1 [p, c, n1], f2
 * [p, c, n2], the [B, C, N] layout the extractor / PVConv produce -- so the
 * registration step matches the devoxelised features in place (same sums,
 * same results as pcr_mutual_nn_match on the transposes). */
pcr_status pcr_mutual_nn_match_cm(const float *f1, const float *f2, int p, int n1, int n2, int c,
                                  int *corr12, int *corr21, int *idx1, int *idx2, int *count,
                                  void *workspace, size_t workspace_bytes, void *stream);

/* ------------------------------------ LRF change_coords (8f f2) ----------
 * models/pvcnn_classify.py:153-184 (rot_invariant_preprocess ==
 * 'change_coords'), one cloud per workgroup, no host round trip.
 * Per cloud: nc = coords - mean (the fp64 mean reduction order is given in
 * oracle/pcr_oracle.c orc_lrf); base_x = the point of largest norm; base_y =
 * the next point in descending-norm rank with norm >= 1e-5 and
 * |<base_x, p/|p|>| < 0.9; Gram-Schmidt, base_z = x cross y; new_coords =
 * basis . nc.  Rank ties go to the lower index.
 *   coords [b,3,n] -> new_coords [b,3,n], basis [b,3,3] (rows x, y, z),
 *   picks [b,2] (base_x, base_y point indices), status [b]: 0 ok, 1 base_x
 *   norm <= 1e-5, 2 no base_y, 3 degenerate Gram-Schmidt.  These are the
 *   reference's asserts; the host shim raises on them. */
pcr_status pcr_lrf_change_coords(const float *coords, int b, int n, float *new_coords,
                                 float *basis, int *picks, int *status, void *stream);

/* --------------------------------- PointNet++ ops (8f f4) ----------------
 * sampling/sampling.cpp:6-58 gather_features_forward / _backward and
 * furthest_point_sampling_forward; interpolate/neighbor_interpolate.cpp:
 * 6-65 three_nearest_neighbors_interpolate_forward / _backward. */
/* features [b,c,n], indices [b,m] -> out [b,c,m] (indices outside [0,n)
 * read 0; the reference reads out of bounds there) */
pcr_status pcr_gather_features_forward(const float *features, const int *indices, int b, int c,
                                       int n, int m, float *out, void *stream);
/* grad_y [b,c,m] -> grad_x [b,c,n] (zeroed here, then scatter-added) */
pcr_status pcr_gather_features_backward(const float *grad_y, const int *indices, int b, int c,
                                        int n, int m, float *grad_x, void *stream);
/* coords [b,3,n] -> indices [b,m].  Tie order as the reference's
 * 512-thread reduction (pcr_fps_key).  workspace: pcr_fps_workspace_size. */
size_t pcr_fps_workspace_size(int b, int n);
pcr_status pcr_furthest_point_sampling(const float *coords, int b, int n, int m, int *indices,
                                       void *workspace, size_t workspace_bytes, void *stream);
/* points [b,3,n], centers [b,3,m], centers_features [b,c,m] ->
 * out [b,c,n], indices [b,3,n], weights [b,3,n] */
pcr_status pcr_three_nn_interpolate_forward(const float *points, const float *centers,
                                            const float *centers_features, int b, int c, int m,
                                            int n, float *out, int *indices, float *weights,
                                            void *stream);
/* grad_y [b,c,n] -> grad_x [b,c,m] (zeroed here, then scatter-added) */
pcr_status pcr_three_nn_interpolate_backward(const float *grad_y, const int *indices,
                                             const float *weights, int b, int c, int n, int m,
                                             float *grad_x, void *stream);

/* ------------------------------------------- normal estimation (8f f3) ----
 * utils/open3d_func.py:77-83 get_normals (Open3D estimate_normals with
 * KDTreeSearchParamRadius(radius) + orient_normals_towards_camera_location()
 * + normalize_normals()), batched on the GPU: points [b,3,n] -> normals
 * [b,3,n] (unit, facing the origin; (0,0,1) with < 3 neighbours),
 * counts [b,n] = neighbours within radius incl. the point (may be NULL).
 * Arithmetic: pcr_estimate_normal of include/pcr_math.h, in fp64. */
pcr_status pcr_estimate_normals(const float *points, int b, int n, double radius, float *normals,
                                int *counts, void *stream);

/* ----------------------------------------- on-disk point rows (8f f3) ----
 * datasets/modelnet40.py:30 np.loadtxt(<sample>.txt, delimiter=',') for the
 * ModelNet40 normal-resampled files ("x,y,z,nx,ny,nz" per line): every
 * value parsed as double, then rounded to float (= loadtxt + astype float32).
 * HOST memory, host code.  pcr_txt_shape counts rows/columns; pcr_read_xyzn_txt
 * fills a row-major [rows, cols] float buffer. */
pcr_status pcr_txt_shape(const char *path, long long *rows, int *cols);
pcr_status pcr_read_xyzn_txt(const char *path, float *out, long long rows, int cols);

/* ------------------------------------------------ native step runner ----
 * `steps` consecutive extractor steps (the pipelined schedule bench.py
 * measures), enqueued from native code: every launch and cross-stream event
 * of every step is issued here, so the host enqueue rate never limits the
 * step rate.  Forked from and joined back into `origin`.
 *   schedule 0: serial, two streams -- s_nbr: Morton sort, KNN selection,
 *               local PPF; s_vox: prep + the fused grid / devox / descriptor
 *               kernel; the single set of buffers (or ring set s).
 *   (schedules 1-5, single-queue-per-stage variants measured in rounds 2-4,
 *   were removed: DESIGN.md 4.)
 *   schedule 6: two independent pipelines per chain and no cross-queue event
 *               inside the run: the voxel chain (prep, means / devox /
 *               descriptor, matching, grid stream) of step s on s_vox (even
 *               s) or `origin` (odd s) with voxel workspace s % 2, the KNN
 *               chain (sort, selection, local PPF) on s_nbr (even) or s_pre
 *               (odd) with KNN workspace s % 2, so every workspace is reused
 *               only on its own queue.  The odd voxel queue starts after step
 *               0's means (one wait per call) so the two grid streams
 *               alternate rather than coincide.  Needs a batch ring of >= 2
 *               sets (consecutive steps write distinct sets); a ring of odd
 *               size that one call wraps orders each set's rewrite behind its
 *               previous step with per-set events (made on first use).
 *   schedule 7: as 6 with three voxel queues (s_vox, origin, s_pre: voxel
 *               workspaces vox_ws[0], vox_ws[1], vox_ws3) and one KNN queue
 *               (s_nbr); needs a ring of >= 3 sets, per-set events when the
 *               ring size is not a multiple of 3.  Schedules 6 / 7 with
 *               match_pairs: each voxel queue matches in its own part (half
 *               / third) of match_ws.
 * Buffers with two entries: schedule 0 uses entry 0; schedules 6 / 7 use
 * knn_ws[q] / vox_ws[q] (+ vox_ws3) as the queue's workspace.
 * desc_steps: [steps][b][c] per-step descriptors, or NULL (then desc).
 *
 * `runner` holds the run's cross-stream events, created once by
 * pcr_runner_create on the current device and reused by every call (NULL:
 * transient events for this call only).  With timed_steps > 0 the runner
 * also brackets the grid-stream kernel (pcr_extractor_voxel_stream) of the
 * min(steps, timed_steps) steps in the middle of each run (pipeline full; fewer after
 * pcr_runner_set_timed) with timing events on its stream;
 * pcr_runner_grid_times waits for them and returns the per-step durations
 * (ms) of the last run -- the dominant kernel's in-step duration.
 *
 * Batch ring (nsets > 0; required by schedules 6 and 7): step s of a call reads its clouds
 * from, and writes every output into, sets[(set0 + s) % nsets] -- a fresh
 * batch per step, as the reference's loaders hand one over per iteration
 * (datasets/deepgmr_mn40.py:71-97, train.py:138-153) -- and the single-set
 * input / output pointers of pcr_extractor_args are ignored (the workspaces
 * stay per queue).  With steps <= nsets every step of a
 * call writes its own set, so after the call (all streams joined back into
 * `origin`) the outputs of every step are readable on `origin`; the next
 * call forks from `origin` after whatever the caller enqueued there, so a
 * consumer enqueued between calls never races the next call's writes.  More
 * steps than sets in one call overwrite set q with step s + nsets. */
typedef struct pcr_runner pcr_runner;
pcr_status pcr_runner_create(int timed_steps, pcr_runner **out);
void pcr_runner_destroy(pcr_runner *runner);
pcr_status pcr_runner_grid_times(pcr_runner *runner, float *ms, int cap, int *count);
/* steps timed by each later run (0..timed_steps of pcr_runner_create; the
 * default is all of them) */
pcr_status pcr_runner_set_timed(pcr_runner *runner, int timed_steps);
typedef struct pcr_extractor_set {
  const float *xyz, *normals, *features;  /* [b,3,n], [b,3,n], [b,c,n] */
  int *knn_idx;                           /* [b,k,n] */
  float *knn_dist;                        /* [b,k,n] or NULL */
  float *local_ppf;                       /* [b,4,k,n] */
  float *norm_coords;                     /* [b,3,n] */
  int *ind, *cnt;                         /* [b,n], [b,r^3] */
  float *grid, *devox, *desc;             /* [b,c,r^3], [b,c,n], [b,c] */
  int *dinds;                             /* [b,8,n] */
  float *dwgts;                           /* [b,8,n] */
  int *corr12, *corr21, *idx1, *idx2, *match_count; /* match_pairs > 0: [P,n] / [P] */
} pcr_extractor_set;
typedef struct pcr_extractor_args {
  int b, n, c, k, r, relative;
  const float *xyz, *normals, *features;  /* [b,3,n], [b,3,n], [b,c,n] */
  int *knn_idx;                           /* [b,k,n] */
  float *knn_dist;                        /* [b,k,n] or NULL */
  float *local_ppf;                       /* [b,4,k,n] */
  float *norm_coords;                     /* [b,3,n] */
  int *ind, *cnt;                         /* [b,n], [b,r^3] */
  float *grid, *devox, *desc;             /* [b,c,r^3], [b,c,n], [b,c] */
  int *dinds[2];                          /* [b,8,n] */
  float *dwgts[2];                        /* [b,8,n] */
  void *knn_ws[2];                        /* pcr_knn_workspace_size(b, n, n) */
  size_t knn_ws_bytes;
  void *vox_ws[2];                        /* pcr_extractor_workspace_size(b, n, c, r) */
  size_t vox_ws_bytes;
  /* registration pairs (BASELINE c4, datasets/deepgmr_mn40.py:71-97,
   * 232-244): match_pairs = P > 0 with b == 2P makes every step also match
   * the devoxelised per-point features of cloud i (source) against cloud
   * P + i (target) by pcr_mutual_nn_match_cm, on the prep stream after the
   * step's devox; outputs [P, n] (count [P]) as that function's. */
  int match_pairs;
  int *corr12, *corr21, *idx1, *idx2, *match_count;
  void *match_ws;                         /* pcr_mutual_nn_workspace_size(P, n, n);
                                             schedules 6 / 7: two / three times
                                             that + 512 B (one part per voxel
                                             queue) */
  size_t match_ws_bytes;
  /* batch ring (see above): nsets sets, step s of the call uses set
   * (set0 + s) % nsets; nsets = 0: the single set above */
  int nsets, set0;
  const pcr_extractor_set *sets;
  /* schedule 7: the third voxel workspace (vox_ws_bytes) */
  void *vox_ws3;
  /* nonzero: the spherical devox + descriptor stay in the means launch
   * (pcr_extractor_voxel_means_devox + pcr_extractor_voxel_stream) even where
   * the grid stream could evaluate them (pcr_extractor_stream_devox_ok); 0
   * (the default): they ride in the grid stream there */
  int devox_in_means;
} pcr_extractor_args;
pcr_status pcr_extractor_run(pcr_runner *runner, const pcr_extractor_args *args, int steps,
                             int schedule, float *desc_steps, void *origin, void *s_nbr,
                             void *s_pre, void *s_vox);

/* ------------------------------------------------------ self tests ------
 * Device evaluation of the shared bit-exact math (include/pcr_math.h) for
 * host-vs-device parity tests.  op: 0 acosf, 1 atanf, 2 sqrtf, 3 x/y,
 * 4 spherical index (x: [3,n] coords, y unused, out_i: index with r=aux). */
pcr_status pcr_selftest_math(int op, const float *x, const float *y, int n, int aux, float *out_f,
                             int *out_i, void *stream);
pcr_status pcr_selftest_math_d(int op, const double *x, const double *y, int n, double *out,
                               void *stream);

#ifdef __cplusplus
}
#endif

#endif /* PCR_AMD_H */
