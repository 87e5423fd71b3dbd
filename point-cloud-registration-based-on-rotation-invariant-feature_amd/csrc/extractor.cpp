// extractor.cpp -- native multi-step runner of the sph-dg extractor forward
// (the bench's pipelined step, include/pcr_amd.h pcr_extractor_run).  Host
// code only: it enqueues the kernels of voxelize.hip / knn_spatial.hip /
// neighbors.hip through their C entry points and chains the streams with HIP
// events, so a Python caller pays one call per S steps instead of a dozen
// ctypes / torch.cuda.Event operations per step.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace pcr {
namespace {

struct Events {
  hipEvent_t e[12] = {};
  int n = 0;
  hipEvent_t make() {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    e[n++] = ev;
    return ev;
  }
  ~Events() {
    for (int i = 0; i < n; i++) (void)hipEventDestroy(e[i]);  // freed once they complete
  }
};

#define PCR_TRY(call)                  \
  do {                                 \
    const pcr_status rc_ = (call);     \
    if (rc_ != PCR_OK) return rc_;     \
  } while (0)
#define PCR_HIP(call, what)                                                      \
  do {                                                                           \
    const hipError_t e_ = (call);                                                \
    if (e_ != hipSuccess) {                                                      \
      set_error("extractor_run: %s failed: %s", what, hipGetErrorString(e_));    \
      return PCR_ERR_LAUNCH;                                                     \
    }                                                                            \
  } while (0)

// diagnostic only (never set in the product): PCR_RUN_SKIP bit mask of
// launches the runner leaves out -- 1 local PPF, 2 grid stream, 4 prep +
// means, 8 sort + selection -- to see which chain bounds the step
static int skip_mask() {
  static const int m = getenv("PCR_RUN_SKIP") ? atoi(getenv("PCR_RUN_SKIP")) : 0;
  return m;
}

// Morton sort of the cloud into KNN workspace q; false when the sorted path
// does not apply (nothing launched; the selection then runs unsorted)
pcr_status knn_sort(const pcr_extractor_args* a, int q, hipStream_t st, bool* sorted) {
  if (skip_mask() & 8) {
    *sorted = true;
    return PCR_OK;
  }
  const pcr_status rc = pcr_knn_prepare(a->xyz, a->b, a->n, a->knn_ws[q], a->knn_ws_bytes, st);
  *sorted = rc == PCR_OK;
  return rc == PCR_ERR_UNSUPPORTED ? PCR_OK : rc;
}

// selection (from KNN workspace q) + local PPF of one step on `st`
pcr_status knn_select_ppf(const pcr_extractor_args* a, int q, bool sorted, hipStream_t st) {
  if (!sorted)  // no sorted path: the one-call selection + PPF
    return pcr_knn_local_ppf(a->xyz, a->normals, a->b, a->n, a->k, a->relative, a->knn_idx,
                             a->knn_dist, a->local_ppf, a->knn_ws[q], a->knn_ws_bytes, st);
  if (!(skip_mask() & 8))
    PCR_TRY(pcr_knn_local_ppf_prepared(a->xyz, a->normals, a->b, a->n, a->k, a->relative,
                                       a->knn_idx, a->knn_dist, nullptr, a->knn_ws[q],
                                       a->knn_ws_bytes, st));
  if (skip_mask() & 1) return PCR_OK;
  return pcr_local_ppf_forward(a->xyz, a->normals, a->xyz, a->normals, a->knn_idx, a->b, a->n,
                               a->n, a->k, 1, a->relative, a->local_ppf, st);
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_extractor_run(const pcr_extractor_args* a, int steps, int schedule,
                                        float* desc_steps, void* origin, void* s_nbr_p,
                                        void* s_pre_p, void* s_vox_p) {
  PCR_REQUIRE(a != nullptr && steps >= 0 && schedule >= 0 && schedule <= 2,
              "extractor_run: invalid arguments");
  PCR_REQUIRE(a->b >= 0 && a->n >= 1 && a->c >= 1 && a->k >= 1 && a->r >= 1,
              "extractor_run: invalid sizes");
  if (steps == 0 || a->b == 0) return PCR_OK;
  const hipStream_t org = as_stream(origin), sn = as_stream(s_nbr_p), sp = as_stream(s_pre_p),
                    sv = as_stream(s_vox_p);
  const int nslots = schedule >= 1 ? 2 : 1;
  for (int q = 0; q < nslots; q++)
    PCR_REQUIRE(a->vox_ws[q] && a->dinds[q] && a->dwgts[q] && a->knn_ws[schedule == 2 ? q : 0],
                "extractor_run: buffer set %d missing", q);
  Events ev;
  hipEvent_t fork = ev.make(), means_done[2] = {ev.make(), ev.make()},
             stream_done[2] = {ev.make(), ev.make()}, join[3] = {ev.make(), ev.make(), ev.make()},
             sort_done[2] = {ev.make(), ev.make()}, sel_done[2] = {ev.make(), ev.make()};
  PCR_REQUIRE(ev.n == 12 && sel_done[1] != nullptr, "extractor_run: event creation failed");
  PCR_HIP(hipEventRecord(fork, org), "fork record");
  for (hipStream_t st : {sn, sp, sv}) PCR_HIP(hipStreamWaitEvent(st, fork, 0), "fork wait");
  const size_t dstride = (size_t)a->b * a->c;
  for (int s = 0; s < steps; s++) {
    float* desc = desc_steps ? desc_steps + (size_t)s * dstride : a->desc;
    bool sorted = false;
    if (schedule == 0) {
      PCR_TRY(knn_sort(a, 0, sn, &sorted));
      PCR_TRY(knn_select_ppf(a, 0, sorted, sn));
      PCR_TRY(pcr_extractor_voxel_stage(a->xyz, a->features, a->b, a->c, a->n, a->r,
                                        a->norm_coords, a->ind, a->cnt, a->grid, a->devox,
                                        a->dinds[0], a->dwgts[0], desc, a->vox_ws[0],
                                        a->vox_ws_bytes, sv));
      continue;
    }
    const int q = s & 1;
    if (schedule == 2) {
      if (s >= 2) PCR_HIP(hipStreamWaitEvent(sp, sel_done[q], 0), "knn slot wait");
      PCR_TRY(knn_sort(a, q, sp, &sorted));
      PCR_HIP(hipEventRecord(sort_done[q], sp), "sort record");
    }
    if (s >= 2) PCR_HIP(hipStreamWaitEvent(sp, stream_done[q], 0), "slot wait");
    if (!(skip_mask() & 4))
      PCR_TRY(pcr_extractor_voxel_prep(a->xyz, a->b, a->n, a->r, a->norm_coords, a->ind,
                                       a->dinds[q], a->dwgts[q], a->vox_ws[q], a->vox_ws_bytes,
                                       sp));
    if (!(skip_mask() & 4))
      PCR_TRY(pcr_extractor_voxel_means_devox(a->features, a->b, a->c, a->n, a->r, a->devox,
                                            a->dinds[q], a->dwgts[q], desc, a->vox_ws[q],
                                            a->vox_ws_bytes, sp));
    PCR_HIP(hipEventRecord(means_done[q], sp), "means record");
    PCR_HIP(hipStreamWaitEvent(sv, means_done[q], 0), "means wait");
    if (!(skip_mask() & 2))
      PCR_TRY(pcr_extractor_voxel_stream(a->b, a->c, a->n, a->r, a->cnt, a->grid, a->vox_ws[q],
                                         a->vox_ws_bytes, sv));
    PCR_HIP(hipEventRecord(stream_done[q], sv), "stream record");
    if (schedule == 2) {
      PCR_HIP(hipStreamWaitEvent(sn, sort_done[q], 0), "sort wait");
      if (sorted) {
        PCR_TRY(pcr_knn_local_ppf_prepared(a->xyz, a->normals, a->b, a->n, a->k, a->relative,
                                           a->knn_idx, a->knn_dist, nullptr, a->knn_ws[q],
                                           a->knn_ws_bytes, sn));
        PCR_HIP(hipEventRecord(sel_done[q], sn), "select record");
        PCR_TRY(pcr_local_ppf_forward(a->xyz, a->normals, a->xyz, a->normals, a->knn_idx, a->b,
                                      a->n, a->n, a->k, 1, a->relative, a->local_ppf, sn));
      } else {
        PCR_TRY(knn_select_ppf(a, q, false, sn));
        PCR_HIP(hipEventRecord(sel_done[q], sn), "select record");
      }
    } else {
      PCR_TRY(knn_sort(a, 0, sn, &sorted));
      PCR_TRY(knn_select_ppf(a, 0, sorted, sn));
    }
  }
  int i = 0;
  for (hipStream_t st : {sn, sp, sv}) {
    PCR_HIP(hipEventRecord(join[i], st), "join record");
    PCR_HIP(hipStreamWaitEvent(org, join[i], 0), "join wait");
    i++;
  }
  return PCR_OK;
}
