// extractor.cpp -- native multi-step runner of the sph-dg extractor forward
// (the bench's pipelined step, include/pcr_amd.h pcr_extractor_run).  Host
// code only: it enqueues the kernels of voxelize.hip / knn_spatial.hip /
// neighbors.hip through their C entry points and chains the streams with HIP
// events, so a Python caller pays one call per S steps instead of a dozen
// ctypes / torch.cuda.Event operations per step.
#include <hip/hip_runtime.h>

#include <vector>

#include "common.hpp"

// the KNN chains of a call's first kS6Head steps wait for step 0's voxel
// means: 20-step calls 366k -> 375k clouds/s (3 interleaved rounds,
// profiles/r05_ab_head_wait.log), 200 steps unchanged
constexpr int kS6Head = 2;

namespace pcr {
namespace {

// the runner's events: created once per runner (per SphExtractor), reused by
// every pcr_extractor_run call.  A wait captures the event's most recent
// record at the time it is enqueued, so re-recording across steps and calls
// keeps the same ordering as fresh events.
constexpr int kSyncEvents = 8;
}  // namespace
}  // namespace pcr

struct pcr_runner {
  int device = 0;
  hipEvent_t sync[pcr::kSyncEvents] = {};
  int timed_cap = 0;              // grid-kernel timing pairs (0: untimed)
  hipEvent_t* t0 = nullptr;       // [timed_cap] before each grid launch
  hipEvent_t* t1 = nullptr;       // [timed_cap] after it
  int timed_last = 0;             // pairs recorded by the last run
  int timed_want = 0;             // steps each run times (<= timed_cap)
  // schedule 6 with an odd batch ring reused inside one call: per-set events
  // (the step that rewrites set t runs on the other queue of its chain)
  std::vector<hipEvent_t> ring_ev;  // [2 * nsets]: voxel chain, KNN chain
  ~pcr_runner() {
    for (hipEvent_t e : sync)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ring_ev)
      if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < timed_cap; i++) {
      if (t0 && t0[i]) (void)hipEventDestroy(t0[i]);
      if (t1 && t1[i]) (void)hipEventDestroy(t1[i]);
    }
    delete[] t0;
    delete[] t1;
  }
};

namespace pcr {
namespace {

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

// The inputs and outputs of one step: the single set of pcr_extractor_args
// (nsets = 0, devox corners alternating with the scratch slot) or the batch
// ring's set (set0 + s) % nsets
struct StepIO {
  const float *xyz, *normals, *features;
  int* knn_idx;
  float *knn_dist, *local_ppf, *norm_coords;
  int *ind, *cnt;
  float *grid, *devox, *desc;
  int* dinds;
  float* dwgts;
  int *corr12, *corr21, *idx1, *idx2, *match_count;
};

StepIO step_io(const pcr_extractor_args* a, int s, int slot) {
  if (a->nsets > 0) {
    const pcr_extractor_set& t = a->sets[(a->set0 + s) % a->nsets];
    return StepIO{t.xyz,  t.normals,     t.features, t.knn_idx, t.knn_dist, t.local_ppf,
                  t.norm_coords, t.ind,  t.cnt,      t.grid,    t.devox,    t.desc,
                  t.dinds, t.dwgts,      t.corr12,   t.corr21,  t.idx1,     t.idx2,
                  t.match_count};
  }
  return StepIO{a->xyz,  a->normals,     a->features,     a->knn_idx, a->knn_dist, a->local_ppf,
                a->norm_coords, a->ind,  a->cnt,          a->grid,    a->devox,    a->desc,
                a->dinds[slot], a->dwgts[slot], a->corr12, a->corr21, a->idx1,     a->idx2,
                a->match_count};
}

// Morton sort of the cloud into KNN workspace q; false when the sorted path
// does not apply (nothing launched; the selection then runs unsorted)
pcr_status knn_sort(const pcr_extractor_args* a, const StepIO& io, int q, hipStream_t st,
                    bool* sorted) {
  const pcr_status rc = pcr_knn_prepare(io.xyz, a->b, a->n, a->knn_ws[q], a->knn_ws_bytes, st);
  *sorted = rc == PCR_OK;
  return rc == PCR_ERR_UNSUPPORTED ? PCR_OK : rc;
}

// selection (from KNN workspace q) + local PPF of one step on `st`
pcr_status knn_select_ppf(const pcr_extractor_args* a, const StepIO& io, int q, bool sorted,
                          hipStream_t st) {
  if (!sorted)  // no sorted path: the one-call selection + PPF
    return pcr_knn_local_ppf(io.xyz, io.normals, a->b, a->n, a->k, a->relative, io.knn_idx,
                             io.knn_dist, io.local_ppf, a->knn_ws[q], a->knn_ws_bytes, st);
  if (io.knn_dist) {  // distances requested: the selection writes in original order
    PCR_TRY(pcr_knn_local_ppf_prepared(io.xyz, io.normals, a->b, a->n, a->k, a->relative,
                                         io.knn_idx, io.knn_dist, nullptr, a->knn_ws[q],
                                         a->knn_ws_bytes, st));
    return pcr_local_ppf_forward(io.xyz, io.normals, io.xyz, io.normals, io.knn_idx, a->b, a->n,
                                 a->n, a->k, 1, a->relative, io.local_ppf, st);
  }
  // selection in sorted query order, the PPF launch writes knn_idx + PPF
  return pcr_knn_select_ppf(io.xyz, io.normals, a->b, a->n, a->k, a->relative, io.knn_idx,
                            io.local_ppf, a->knn_ws[q], a->knn_ws_bytes, st);
}

// the step's registration matching (source clouds [0, P) against targets
// [P, 2P)) on the devox features the step just wrote; nparts > 1: schedules
// 6 / 7, whose voxel queues each match in their own part of the workspace
pcr_status match_pairs(const pcr_extractor_args* a, const StepIO& io, hipStream_t st,
                       int part = 0, int nparts = 1) {
  if (a->match_pairs <= 0) return PCR_OK;
  const int P = a->match_pairs;
  const float* src = io.devox;
  const float* tgt = io.devox + (size_t)P * a->c * a->n;
  void* ws = a->match_ws;
  size_t bytes = a->match_ws_bytes;
  if (nparts > 1) {
    bytes = a->match_ws_bytes / nparts / 256 * 256;
    ws = (char*)a->match_ws + (size_t)part * bytes;
  }
  return pcr_mutual_nn_match_cm(src, tgt, P, a->n, a->n, a->c, io.corr12, io.corr21, io.idx1,
                                io.idx2, io.match_count, ws, bytes, st);
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_runner_create(int timed_steps, pcr_runner** out) {
  PCR_REQUIRE(out != nullptr && timed_steps >= 0 && timed_steps <= (1 << 16),
              "runner_create: invalid arguments");
  *out = nullptr;
  pcr_runner* rn = new pcr_runner();
  if (hipGetDevice(&rn->device) != hipSuccess) {
    delete rn;
    set_error("runner_create: no HIP device");
    return PCR_ERR_LAUNCH;
  }
  bool ok = true;
  // the sync events only order the runner's streams on this device (every
  // kernel's own dispatch packet carries its acquire / release), so their
  // system-scope fences -- host visibility, cache write-backs at every record
  // -- are dropped: c2 A/B on one box, 3 interleaved rounds, 0.0971 -> 0.0953
  // ms per step (profiles/r04_ab_events.log); hipEventReleaseToDevice alone
  // measured no better than the default.  The caller's stream is joined
  // after the run with these events, and the host synchronises through its
  // own (system-scope) events.
  const unsigned scope = hipEventDisableSystemFence;
  for (int i = 0; i < kSyncEvents; i++)
    ok = ok && hipEventCreateWithFlags(&rn->sync[i], hipEventDisableTiming | scope) == hipSuccess;
  // timing events: device-scope release (hipEventReleaseToDevice: more
  // precise timings, no system-scope write-back inside the timed kernel's
  // bracket)
  const unsigned tscope = hipEventReleaseToDevice;
  if (ok && timed_steps > 0) {
    rn->t0 = new hipEvent_t[timed_steps]();
    rn->t1 = new hipEvent_t[timed_steps]();
    rn->timed_cap = timed_steps;
    rn->timed_want = timed_steps;
    for (int i = 0; i < timed_steps && ok; i++)
      ok = hipEventCreateWithFlags(&rn->t0[i], tscope) == hipSuccess &&
           hipEventCreateWithFlags(&rn->t1[i], tscope) == hipSuccess;
  }
  if (!ok) {
    delete rn;
    set_error("runner_create: event creation failed");
    return PCR_ERR_LAUNCH;
  }
  *out = rn;
  return PCR_OK;
}

extern "C" void pcr_runner_destroy(pcr_runner* rn) { delete rn; }

extern "C" pcr_status pcr_runner_set_timed(pcr_runner* rn, int timed_steps) {
  PCR_REQUIRE(rn != nullptr && timed_steps >= 0 && timed_steps <= rn->timed_cap,
              "runner_set_timed: %d outside [0, %d]", timed_steps, rn ? rn->timed_cap : 0);
  rn->timed_want = timed_steps;
  return PCR_OK;
}

extern "C" pcr_status pcr_runner_grid_times(pcr_runner* rn, float* ms, int cap, int* count) {
  PCR_REQUIRE(rn != nullptr && ms != nullptr && count != nullptr, "runner_grid_times: NULL");
  const int m = rn->timed_last < cap ? rn->timed_last : cap;
  for (int i = 0; i < m; i++) {
    PCR_HIP(hipEventSynchronize(rn->t1[i]), "timing sync");
    PCR_HIP(hipEventElapsedTime(&ms[i], rn->t0[i], rn->t1[i]), "elapsed");
  }
  *count = m;
  return PCR_OK;
}

extern "C" pcr_status pcr_extractor_run(pcr_runner* runner, const pcr_extractor_args* a,
                                        int steps, int schedule, float* desc_steps, void* origin,
                                        void* s_nbr_p, void* s_pre_p, void* s_vox_p) {
  PCR_REQUIRE(a != nullptr && steps >= 0 && (schedule == 0 || schedule == 6 || schedule == 7),
              "extractor_run: invalid arguments (schedule 0, 6 or 7)");
  PCR_REQUIRE(a->b >= 0 && a->n >= 1 && a->c >= 1 && a->k >= 1 && a->r >= 1,
              "extractor_run: invalid sizes");
  PCR_REQUIRE(a->match_pairs <= 0 || a->b == 2 * a->match_pairs,
              "extractor_run: match_pairs %d needs b == 2 * match_pairs (b = %d)",
              a->match_pairs, a->b);
  if (steps == 0 || a->b == 0) return PCR_OK;
  const hipStream_t org = as_stream(origin), sn = as_stream(s_nbr_p), sp = as_stream(s_pre_p),
                    sv = as_stream(s_vox_p);
  PCR_REQUIRE(a->nsets >= 0 && (a->nsets == 0 || (a->sets && a->set0 >= 0)),
              "extractor_run: a batch ring needs sets and set0 >= 0");
  // schedules 6 / 7: nvq voxel queues and nkq KNN queues, each running a
  // whole chain of every nvq-th / nkq-th step
  const int nvq = schedule == 7 ? 3 : 2, nkq = schedule == 7 ? 1 : 2;
  const bool multi = schedule >= 6;
  const int nvws = multi ? nvq : 1, nkws = multi ? nkq : 1;  // workspaces in use
  // consecutive steps are written from different queues: they need distinct
  // output sets (the c5 voxel path counts into cnt with atomics)
  PCR_REQUIRE(!multi || a->nsets >= nvq,
              "extractor_run: schedule %d needs a batch ring of at least %d sets", schedule,
              nvq);
  // the voxel queues match at once: each part of the matching workspace
  // must hold one matching
  PCR_REQUIRE(!multi || a->match_pairs <= 0 ||
                  a->match_ws_bytes / nvq / 256 * 256 >=
                      pcr_mutual_nn_workspace_size(a->match_pairs, a->n, a->n),
              "extractor_run: schedule %d with match_pairs needs a matching workspace of "
              "%d x pcr_mutual_nn_workspace_size (plus 512 B)", schedule, nvq);
  PCR_REQUIRE(schedule != 7 || a->vox_ws3 != nullptr,
              "extractor_run: schedule 7 needs the third voxel workspace (vox_ws3)");
  void* const vws[3] = {a->vox_ws[0], a->vox_ws[1], a->vox_ws3};
  for (int q = 0; q < nvws; q++)
    PCR_REQUIRE(vws[q] != nullptr, "extractor_run: voxel workspace %d missing", q);
  for (int q = 0; q < nkws; q++)
    PCR_REQUIRE(a->knn_ws[q] != nullptr, "extractor_run: KNN workspace %d missing", q);
  PCR_REQUIRE(a->nsets > 0 || (a->dinds[0] && a->dwgts[0]),
              "extractor_run: devox corner buffers missing");
  for (int t = 0; t < a->nsets; t++)
    PCR_REQUIRE(a->sets[t].xyz && a->sets[t].normals && a->sets[t].features &&
                    a->sets[t].knn_idx && a->sets[t].local_ppf && a->sets[t].grid &&
                    a->sets[t].devox && a->sets[t].dinds && a->sets[t].dwgts,
                "extractor_run: ring set %d incomplete", t);
  // no runner: a transient one (events created and destroyed in this call;
  // hipEventDestroy of a pending event is deferred until it completes)
  pcr_runner* tmp = nullptr;
  if (runner == nullptr) {
    PCR_TRY(pcr_runner_create(0, &tmp));
    runner = tmp;
  }
  struct Owned {
    pcr_runner* p;
    ~Owned() { delete p; }
  } owned{tmp};
  pcr_runner* const rn = runner;
  rn->timed_last = !multi ? 0 : steps < rn->timed_want ? steps : rn->timed_want;
  // the timed_last steps in the MIDDLE of the run are timed: the pipeline
  // is full there (the last steps' grid kernels run beside a draining
  // pipeline: at c2 under schedule 6 ~64 us against ~102 us in steady state)
  const int t_first = (steps - rn->timed_last) / 2;
  hipEvent_t* e = rn->sync;
  hipEvent_t fork = e[0], means_done[2] = {e[1], e[2]}, join[3] = {e[5], e[6], e[7]};
  // schedules 6 / 7 over a ring that one call wraps onto other queues
  // (nsets not a multiple of the queue count): per-set events, made once
  // per ring size (the first call, outside any timed region)
  const bool ring_wait = multi && a->nsets > 0 && steps > a->nsets &&
                         (a->nsets % nvq != 0 || a->nsets % nkq != 0);
  if (ring_wait && rn->ring_ev.size() != (size_t)(2 * a->nsets)) {
    for (hipEvent_t ev : rn->ring_ev)
      if (ev) (void)hipEventDestroy(ev);
    rn->ring_ev.assign(2 * a->nsets, nullptr);
    const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
    for (hipEvent_t& ev : rn->ring_ev) PCR_HIP(hipEventCreateWithFlags(&ev, fl), "ring event");
  }
  PCR_HIP(hipEventRecord(fork, org), "fork record");
  for (hipStream_t st : {sn, sp, sv}) PCR_HIP(hipStreamWaitEvent(st, fork, 0), "fork wait");
  const size_t dstride = (size_t)a->b * a->c;
  for (int s = 0; s < steps; s++) {
    const StepIO io = step_io(a, s, 0);
    float* desc = desc_steps ? desc_steps + (size_t)s * dstride : io.desc;
    bool sorted = false;
    if (schedule == 0) {
      PCR_TRY(knn_sort(a, io, 0, sn, &sorted));
      PCR_TRY(knn_select_ppf(a, io, 0, sorted, sn));
      PCR_TRY(pcr_extractor_voxel_stage(io.xyz, io.features, a->b, a->c, a->n, a->r,
                                        io.norm_coords, io.ind, io.cnt, io.grid, io.devox,
                                        io.dinds, io.dwgts, desc, a->vox_ws[0],
                                        a->vox_ws_bytes, sv));
      PCR_TRY(match_pairs(a, io, sv));
      continue;
    }
    // independent pipelines per chain, no cross-queue events: the voxel
    // chain (prep, means / devox, match, grid stream) of step s on voxel
    // queue s % nvq with voxel workspace s % nvq, the KNN chain (sort,
    // selection, local PPF) on KNN queue s % nkq with KNN workspace s % nkq;
    // every workspace is reused only by its own queue.  Schedule 6: voxel
    // queues {s_vox, origin}, KNN queues {s_nbr, s_pre}; schedule 7: voxel
    // queues {s_vox, origin, s_pre}, KNN queue s_nbr
    const hipStream_t vqs[3] = {sv, org, sp}, kqs[2] = {sn, sp};
    const int iv = s % nvq, ik = s % nkq;
    const hipStream_t vq = vqs[iv], kq = kqs[ik];
    void* const vw6 = vws[iv];
    const int t = a->nsets > 0 ? (a->set0 + s) % a->nsets : 0;
    hipEvent_t* const rv = ring_wait ? rn->ring_ev.data() : nullptr;
    if (rv && s >= a->nsets) {  // set t last written on the other queues
      PCR_HIP(hipStreamWaitEvent(vq, rv[2 * t], 0), "ring wait");
      PCR_HIP(hipStreamWaitEvent(kq, rv[2 * t + 1], 0), "ring wait");
    }
    auto knn_part = [&]() -> pcr_status {
      PCR_TRY(knn_sort(a, io, ik, kq, &sorted));
      return knn_select_ppf(a, io, ik, sorted, kq);
    };
    auto vox_part = [&]() -> pcr_status {
      // voxel queue i > 0 starts after step i - 1's means, so the queues'
      // grid streams take turns rather than coincide (aligned, they fight
      // for HBM and then leave it idle together)
      if (s >= 1 && s < nvq) PCR_HIP(hipStreamWaitEvent(vq, means_done[s - 1], 0), "offset wait");
      PCR_TRY(pcr_extractor_voxel_prep(io.xyz, a->b, a->n, a->r, io.norm_coords, io.ind,
                                       io.dinds, io.dwgts, vw6, a->vox_ws_bytes, vq));
      // c2-sized clouds: the devox + descriptor ride in the grid stream (its
      // means are in LDS there), so the means launch reads no corner data
      // (c2 390k -> 405-408k clouds/s).  With pair matching, which reads the
      // devox, the matching then runs behind the stream on the same queue:
      // since round 6 (matching of four launches, schedule 6) 337-343k
      // against 326-330k clouds/s with the devox in the means launch and the
      // matching ahead of the stream (profiles/r06_ab_pairs_stream_devox.log)
      const bool dv = !a->devox_in_means && pcr_extractor_stream_devox_ok(a->n, a->c, a->r);
      if (dv)
        PCR_TRY(pcr_extractor_voxel_means(io.features, a->b, a->c, a->n, a->r, vw6,
                                          a->vox_ws_bytes, vq));
      else
        PCR_TRY(pcr_extractor_voxel_means_devox(io.features, a->b, a->c, a->n, a->r, io.devox,
                                                io.dinds, io.dwgts, desc, vw6, a->vox_ws_bytes,
                                                vq));
      if (s < nvq - 1) PCR_HIP(hipEventRecord(means_done[s], vq), "offset record");
      if (!dv) PCR_TRY(match_pairs(a, io, vq, iv, nvq));
      const bool timed = s >= t_first && s < t_first + rn->timed_last;
      if (timed) PCR_HIP(hipEventRecord(rn->t0[s - t_first], vq), "timing record");
      if (dv)
        PCR_TRY(pcr_extractor_voxel_stream_devox(a->b, a->c, a->n, a->r, io.cnt, io.grid,
                                                 io.devox, io.dwgts, desc, vw6,
                                                 a->vox_ws_bytes, vq));
      else
        PCR_TRY(pcr_extractor_voxel_stream(a->b, a->c, a->n, a->r, io.cnt, io.grid, vw6,
                                           a->vox_ws_bytes, vq));
      if (timed) PCR_HIP(hipEventRecord(rn->t1[s - t_first], vq), "timing record");
      if (dv) PCR_TRY(match_pairs(a, io, vq, iv, nvq));
      return PCR_OK;
    };
    // the head of a call: the KNN chains of the first kS6Head steps wait for
    // step 0's voxel means, so prep + means of step 0 get the chip first and
    // its grid stream starts sooner (the call's fill)
    if (s < kS6Head) {
      if (s == 0) PCR_TRY(vox_part());
      PCR_HIP(hipStreamWaitEvent(kq, means_done[0], 0), "head wait");
      PCR_TRY(knn_part());
      if (s != 0) PCR_TRY(vox_part());
    } else {
      PCR_TRY(knn_part());
      PCR_TRY(vox_part());
    }
    if (rv && s + a->nsets < steps) {
      PCR_HIP(hipEventRecord(rv[2 * t], vq), "ring record");
      PCR_HIP(hipEventRecord(rv[2 * t + 1], kq), "ring record");
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
