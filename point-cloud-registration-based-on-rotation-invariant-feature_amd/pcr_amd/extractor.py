"""Fused sph-dg extractor forward: the north-star hot path as one step.

One step over a batch of clouds (xyz [B,3,N], normals [B,3,N], point
features [B,C,N], all resident on the GPU):

  front (stream P): Morton sort of the cloud for KNN; Spherical_Voxelization
      normalisation (PVCNN/modules/spherical_vox.py:16-20) + voxel index /
      occupancy / devox corners (prep)
  neighbours (stream A): self-KNN (k) -> local PPF [B,4,k,N]
      = knn_forward_cuda + the model's local-PPF block
        (PVCNN/models/pvcnn_classify.py:252-269), one kernel
  grid (stream B): spherical_avg_voxelize's dense grid [B,C,r^3] + cnt, then
      spherical_trilinear_devoxelize of that grid ([B,C,N] + inds/wgts) +
      per-cloud descriptor (max over points) [B,C], reading only the 80
      corner voxels per channel every spherical corner lies in (clouds of
      more than 4096 points: the devox re-forms the voxel means on stream C)

The streams are forked from and joined back to the caller's stream.
``forward()`` enqueues one step from Python; ``capture()`` records one step
into a hipGraph; ``run_native()`` has the library (pcr_extractor_run) enqueue
S consecutive steps with no join between them on alternating buffer sets, so
step i+1's front stages overlap step i's back stages -- the product schedule
bench.py measures.
"""
import ctypes

import torch

from . import _lib
from .ops import _ptr


class SphExtractor:
    def __init__(self, batch, npoints, channels, k, resolution, device="cuda", relative=True,
                 with_dist=False, split_ppf=True, stream_devox=True):
        # stream_devox: the split voxel stage evaluates the devox inside the
        # grid stream where it applies (<= 1024 points); False keeps it in the
        # means launch, in the eager / pipelined paths and in the native
        # runner (pcr_extractor_args.devox_in_means)
        self.stream_devox = stream_devox
        self.b, self.n, self.c, self.k, self.r = batch, npoints, channels, k, resolution
        self.relative = relative
        self.split_ppf = split_ppf
        self.device = torch.device(device)
        b, n, c, r = batch, npoints, channels, resolution
        r3 = r * r * r
        dev = self.device
        e = torch.empty
        self.knn_idx = e((b, k, n), dtype=torch.int32, device=dev)
        self.knn_dist = e((b, k, n), dtype=torch.float32, device=dev) if with_dist else None
        self.local_ppf = e((b, 4, k, n), dtype=torch.float32, device=dev)
        self.norm_coords = e((b, 3, n), dtype=torch.float32, device=dev)
        self.ind = e((b, n), dtype=torch.int32, device=dev)
        self.cnt = e((b, r3), dtype=torch.int32, device=dev)
        self.grid = e((b, c, r3), dtype=torch.float32, device=dev)
        self.devox = e((b, c, n), dtype=torch.float32, device=dev)
        self.dinds = e((b, 8, n), dtype=torch.int32, device=dev)
        self.dwgts = e((b, 8, n), dtype=torch.float32, device=dev)
        self.desc = e((b, c), dtype=torch.float32, device=dev)
        lib = _lib.load()
        self.ws = e(max(256, lib.pcr_extractor_workspace_size(b, n, c, r)), dtype=torch.uint8,
                    device=dev)
        self.knn_ws = e(max(256, lib.pcr_knn_workspace_size(b, n, n)), dtype=torch.uint8,
                        device=dev)
        self.s_pre = torch.cuda.Stream(device=dev)
        self.s_nbr = torch.cuda.Stream(device=dev)
        self.s_vox = torch.cuda.Stream(device=dev)
        self.s_dev = torch.cuda.Stream(device=dev)
        self.graph = None
        self._runner, self._runner_cap = None, 0
        self._static_in = None
        self._set1 = None
        self._vsep, self._vset1 = False, None
        self._ppf1 = None
        self._args, self._args_key = None, None
        self._ring_seen = None  # (batch tuples, match, args key) of the last run_ring

    # ---------------------------------------------------------------- stages
    # Buffers a later stage of the same step reads (the two workspaces and the
    # devox corners) come in two sets, so a pipelined caller can run step i+1's
    # front stages while step i's back stages still read set i % 2.
    def _set(self, slot):
        if slot == 0:
            return self.knn_ws, self.ws, self.dinds, self.dwgts, self.knn_idx
        if self._set1 is None:
            e = torch.empty_like
            self._set1 = (e(self.knn_ws), e(self.ws), e(self.dinds), e(self.dwgts),
                          e(self.knn_idx))
            self._order_new_buffers()
        return self._set1

    def _order_new_buffers(self):
        """Buffers made lazily come from the current stream's pool, possibly
        a block freed with kernels still pending on that stream; the
        extractor's streams, which write them, wait for the current stream
        first."""
        cur = torch.cuda.current_stream(self.device)
        for st in (self.s_pre, self.s_nbr, self.s_vox, self.s_dev):
            st.wait_stream(cur)

    def _ppf(self, slot):
        """The local PPF output of index set `slot` (set 1's is made on first
        use: only the train-step pipeline alternates PPF outputs)."""
        if slot == 0:
            return self.local_ppf
        if self._ppf1 is None:
            self._ppf1 = torch.empty_like(self.local_ppf)
            self._order_new_buffers()
        return self._ppf1

    def _vset(self, slot):
        """The voxel outputs of slot `slot`: (norm_coords, ind, devox, desc).
        One set unless a pipeline runs the next batch's voxel head ahead
        (pipelined_steps(voxel_ahead=True)): then slot 1 has its own."""
        if slot == 0 or not self._vsep:
            return self.norm_coords, self.ind, self.devox, self.desc
        if self._vset1 is None:
            e = torch.empty_like
            self._vset1 = (e(self.norm_coords), e(self.ind), e(self.devox), e(self.desc))
            self._order_new_buffers()
        return self._vset1

    def neighbor_stage(self, xyz, normals, stream):
        """Sort + select + PPF in one call (the eager, unsplit path)."""
        _lib.check(_lib.load().pcr_knn_local_ppf(
            _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative),
            _ptr(self.knn_idx), _ptr(self.knn_dist), _ptr(self.local_ppf), _ptr(self.knn_ws),
            self.knn_ws.numel(), stream), "knn_local_ppf")

    def knn_sort(self, xyz, stream, slot=0):
        """Morton sort into workspace set `slot`; False when the sorted path
        does not apply (then knn_select falls back to the one-call path)."""
        kws = self._set(slot)[0]
        rc = _lib.load().pcr_knn_prepare(_ptr(xyz), self.b, self.n, _ptr(kws), kws.numel(),
                                         stream)
        if rc == -3:  # PCR_ERR_UNSUPPORTED, nothing launched
            return False
        _lib.check(rc, "knn_prepare")
        return True

    def knn_select(self, xyz, normals, stream, slot=0, sorted_ok=True, ppf=True, events=None):
        """Selection (+ local PPF unless ppf=False) into index set `slot`.
        events: (ev0, ev1) torch.cuda.Events recorded on `stream` (a
        torch.cuda.Stream) around the selection launch alone."""
        kws, idx = self._set(slot)[0], self._set(slot)[4]
        ppf_out = self._ppf(slot)
        torch_stream = stream if isinstance(stream, torch.cuda.Stream) else None
        if torch_stream is not None:
            stream = torch_stream.cuda_stream
        if torch_stream is None:
            events = None  # events are recorded on a torch.cuda.Stream
        if not sorted_ok:
            _lib.check(_lib.load().pcr_knn_local_ppf(
                _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative),
                _ptr(idx), _ptr(self.knn_dist), _ptr(ppf_out), _ptr(kws),
                kws.numel(), stream), "knn_local_ppf")
            return
        lib = _lib.load()
        if self.split_ppf and ppf and self.knn_dist is None and events is not None:
            # the same two launches with timing events around the selection
            ev0, ev1 = events
            ev0.record(torch_stream)
            rs = lib.pcr_knn_select_sorted(_ptr(xyz), self.b, self.n, self.k, _ptr(kws),
                                           kws.numel(), stream)
            ev1.record(torch_stream)
            if rs == 0:
                _lib.check(lib.pcr_knn_ppf_sorted(
                    _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative),
                    _ptr(idx), _ptr(ppf_out), _ptr(kws), kws.numel(), stream),
                    "knn_ppf_sorted")
                return
            if rs != -3:  # PCR_ERR_UNSUPPORTED: nothing launched
                _lib.check(rs, "knn_select_sorted")
            # the sorted path does not apply: the events are recorded again
            # around the fallback below (its selection + PPF), so they never
            # read ~0 for a launch that ran outside them
            ev0.record(torch_stream)
        else:
            events = None
        if self.split_ppf and ppf and self.knn_dist is None:
            # selection in sorted query order + the PPF launch that writes
            # knn_idx and the PPF (pcr_knn_select_ppf)
            _lib.check(lib.pcr_knn_select_ppf(
                _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative), _ptr(idx),
                _ptr(ppf_out), _ptr(kws), kws.numel(), stream), "knn_select_ppf")
            if events is not None:
                events[1].record(torch_stream)
            return
        _lib.check(lib.pcr_knn_local_ppf_prepared(
            _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative),
            _ptr(idx), _ptr(self.knn_dist), None if self.split_ppf else
            _ptr(ppf_out), _ptr(kws), kws.numel(), stream), "knn_local_ppf_prepared")
        if self.split_ppf and ppf:
            # PPF as its own launch: one thread per (slot, point), coalesced
            _lib.check(lib.pcr_local_ppf_forward(
                _ptr(xyz), _ptr(normals), _ptr(xyz), _ptr(normals), _ptr(idx), self.b,
                self.n, self.n, self.k, 1, int(self.relative), _ptr(ppf_out), stream),
                "local_ppf_forward")

    def voxel_stage(self, xyz, features, stream, desc=None):
        """prep + the fused grid / devox / descriptor kernel, one call."""
        d = self.desc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_stage(
            _ptr(xyz), _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.norm_coords),
            _ptr(self.ind), _ptr(self.cnt), _ptr(self.grid), _ptr(self.devox), _ptr(self.dinds),
            _ptr(self.dwgts), _ptr(d), _ptr(self.ws), self.ws.numel(), stream),
            "extractor_voxel_stage")

    def voxel_prep(self, xyz, stream, slot=0):
        _, ws, dinds, dwgts, _ = self._set(slot)
        nc, ind, _, _ = self._vset(slot)
        _lib.check(_lib.load().pcr_extractor_voxel_prep(
            _ptr(xyz), self.b, self.n, self.r, _ptr(nc), _ptr(ind),
            _ptr(dinds), _ptr(dwgts), _ptr(ws), ws.numel(), stream), "extractor_voxel_prep")

    def voxel_grid(self, features, stream, slot=0):
        """The dominant kernel (vox_grid_kernel<1>: means -> dense grid + cnt)."""
        ws = self._set(slot)[1]
        _lib.check(_lib.load().pcr_extractor_voxel_grid(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.cnt), _ptr(self.grid),
            _ptr(ws), ws.numel(), stream), "extractor_voxel_grid")

    def voxel_grid_devox(self, features, stream, desc=None, slot=0):
        """The dominant kernel of the default step (vox_grid_kernel<3>: dense
        grid + cnt, devox + descriptor from the same LDS means)."""
        _, ws, dinds, dwgts, _ = self._set(slot)
        d = self.desc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_grid_devox(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.cnt), _ptr(self.grid),
            _ptr(self.devox), _ptr(dinds), _ptr(dwgts), _ptr(d), _ptr(ws),
            ws.numel(), stream), "extractor_voxel_grid_devox")

    def voxel_means_devox(self, features, stream, desc=None, slot=0):
        """Voxel means of the occupied segments into the workspace + devox +
        descriptor (the first half of the split voxel stage)."""
        _, ws, dinds, dwgts, _ = self._set(slot)
        _, _, devox, vdesc = self._vset(slot)
        d = vdesc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_means_devox(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(devox), _ptr(dinds),
            _ptr(dwgts), _ptr(d), _ptr(ws), ws.numel(), stream), "extractor_voxel_means_devox")

    def voxel_means(self, features, stream, slot=0):
        """Voxel means of the occupied segments into the workspace only (the
        devox + descriptor then ride in voxel_stream_devox)."""
        ws = self._set(slot)[1]
        _lib.check(_lib.load().pcr_extractor_voxel_means(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(ws), ws.numel(), stream),
            "extractor_voxel_means")

    def voxel_stream_devox(self, stream, desc=None, slot=0):
        """The dense grid + cnt, devox and descriptor from the workspace means
        (pcr_extractor_voxel_stream_devox: each grid workgroup reads the
        cloud's corner data once)."""
        _, ws, _, dwgts, _ = self._set(slot)
        _, _, devox, vdesc = self._vset(slot)
        d = vdesc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_stream_devox(
            self.b, self.c, self.n, self.r, _ptr(self.cnt), _ptr(self.grid), _ptr(devox),
            _ptr(dwgts), _ptr(d), _ptr(ws), ws.numel(), stream), "extractor_voxel_stream_devox")

    def voxel_stream(self, stream, slot=0):
        """The dense grid + cnt from the workspace means (the dominant,
        HBM-bound kernel of the split voxel stage)."""
        ws = self._set(slot)[1]
        _lib.check(_lib.load().pcr_extractor_voxel_stream(
            self.b, self.c, self.n, self.r, _ptr(self.cnt), _ptr(self.grid), _ptr(ws),
            ws.numel(), stream), "extractor_voxel_stream")

    def grid_devox(self, stream, desc=None, slot=0):
        """Devox + descriptor from the dense grid (after voxel_grid on the
        same stream): the 80 corner voxels per channel staged in LDS."""
        _, _, dinds, dwgts, _ = self._set(slot)
        _, _, devox, vdesc = self._vset(slot)
        d = vdesc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_grid_devox(
            _ptr(self.grid), _ptr(dinds), _ptr(dwgts), self.b, self.c, self.n, self.r,
            _ptr(devox), _ptr(d), stream), "extractor_grid_devox")

    def voxel_devox(self, features, stream, desc=None, slot=0):
        _, ws, dinds, dwgts, _ = self._set(slot)
        _, _, devox, vdesc = self._vset(slot)
        d = vdesc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_devox(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(devox), _ptr(dinds),
            _ptr(dwgts), _ptr(d), _ptr(ws), ws.numel(), stream), "extractor_voxel_devox")

    def _check_inputs(self, xyz, normals, features):
        for t, name in ((xyz, "xyz"), (normals, "normals"), (features, "features")):
            if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
                raise RuntimeError("%s must be a contiguous float CUDA tensor" % name)
        if tuple(xyz.shape) != (self.b, 3, self.n) or tuple(features.shape) != (self.b, self.c,
                                                                                  self.n):
            raise RuntimeError("input shape does not match the extractor configuration")

    def _streams(self):
        return (self.s_pre, self.s_nbr, self.s_vox, self.s_dev)

    def _fork(self):
        cur = torch.cuda.current_stream(self.device)
        for st in self._streams():
            st.wait_stream(cur)
        return cur

    def _join(self, cur):
        for st in self._streams():
            cur.wait_stream(st)

    def enqueue(self, xyz, normals, features, desc=None, slot=0, reuse=None, events=False):
        """Enqueue one step on the extractor's streams, no fork/join:
          s_pre: KNN Morton sort, voxel prep (both small, one workgroup per cloud)
          s_nbr: KNN selection + local PPF      (after the sort)
          s_vox: voxel grid, then devox + descriptor from that grid (after prep)
        `reuse` = events after which the previous users of buffer set `slot`
        are done (s_pre waits for them before overwriting it).  With
        `events`, returns this step's events on buffer set `slot`."""
        if reuse:
            for ev in reuse:
                self.s_pre.wait_event(ev)
        sorted_ok = self.knn_sort(xyz, self.s_pre.cuda_stream, slot)
        e_sort = torch.cuda.Event()
        e_sort.record(self.s_pre)
        self.voxel_prep(xyz, self.s_pre.cuda_stream, slot)
        e_prep = torch.cuda.Event()
        e_prep.record(self.s_pre)
        self.s_nbr.wait_event(e_sort)
        self.knn_select(xyz, normals, self.s_nbr.cuda_stream, slot, sorted_ok)
        self.s_vox.wait_event(e_prep)
        self.voxel_grid(features, self.s_vox.cuda_stream, slot)
        if self.n <= 4096:
            # the devox reads the 80 corner voxels per channel of the grid
            # just written (same stream)
            self.grid_devox(self.s_vox.cuda_stream, desc, slot)
        else:
            self.s_dev.wait_event(e_prep)
            self.voxel_devox(features, self.s_dev.cuda_stream, desc, slot)
        if not events:
            return None
        evs = []
        for st in (self.s_nbr, self.s_vox, self.s_dev):
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
        return evs

    def forward(self, xyz, normals, features):
        """Enqueue one step, forked from and joined back to the current stream."""
        self._check_inputs(xyz, normals, features)
        cur = self._fork()
        self.enqueue(xyz, normals, features)
        self._join(cur)
        return self.outputs()

    # ------------------------------------------------- train-step pipeline
    def enqueue_neighbors(self, xyz, normals, slot, after=None, events=None):
        """Self-KNN (Morton sort + selection) + local PPF of one batch on
        s_nbr into index set `slot` (its knn_idx / local_ppf).  `after`: an
        event recorded once the set's previous consumer is done with it.
        events: (ev0, ev1) around the selection launch.  Returns the event
        this batch's consumer waits on."""
        if after is not None:
            self.s_nbr.wait_event(after)
        sorted_ok = self.knn_sort(xyz, self.s_nbr.cuda_stream, slot)
        self.knn_select(xyz, normals, self.s_nbr if events is not None else
                        self.s_nbr.cuda_stream, slot, sorted_ok, events=events)
        ev = torch.cuda.Event()
        ev.record(self.s_nbr)
        return ev

    def enqueue_voxels(self, xyz, features, stream, slot=0, desc=None):
        """The voxel side of one batch on `stream`: normalisation + voxel
        index + devox corners (prep), the dense grid + cnt, then devox +
        descriptor (from the grid's 80 corner voxels per channel, or from
        the re-formed means past 4096 points).  Clouds of <= 2048 points on
        grids the streaming kernel takes (r^3 a multiple of 2048, <= 32^3)
        use the split stage: voxel means + devox + descriptor in one launch,
        then the dense grid streamed from the compact means (c3: 0.60 +
        0.16 ms -> see DESIGN.md 4)."""
        if self._split_voxels():
            self.voxel_head(xyz, features, stream, slot, desc)
            self.voxel_tail(stream, slot, desc)
            return
        self.voxel_prep(xyz, stream, slot)
        self.voxel_grid(features, stream, slot)
        if self.n <= 4096:
            self.grid_devox(stream, desc, slot)
        else:
            self.voxel_devox(features, stream, desc, slot)

    def _split_voxels(self):
        """Clouds of <= 2048 points on grids the streaming kernel takes (r^3 a
        multiple of 2048, <= 32^3): the split voxel stage (head: prep +
        means; tail: the dense-grid stream)."""
        r3 = self.r ** 3
        return self.n <= 2048 and r3 % 2048 == 0 and r3 <= 32768

    def _stream_devox(self):
        return self.stream_devox and bool(
            _lib.load().pcr_extractor_stream_devox_ok(self.n, self.c, self.r))

    def voxel_head(self, xyz, features, stream, slot=0, desc=None):
        """The split voxel stage's head: prep, then the voxel means (with the
        devox + descriptor unless they ride in the grid stream)."""
        self.voxel_prep(xyz, stream, slot)
        if self._stream_devox():
            self.voxel_means(features, stream, slot)
        else:
            self.voxel_means_devox(features, stream, desc, slot)

    def voxel_tail(self, stream, slot=0, desc=None):
        """The split voxel stage's tail: the dense grid + cnt streamed from the
        head's means (with the devox + descriptor for <= 1024-point clouds,
        DESIGN.md 4.5)."""
        if self._stream_devox():
            self.voxel_stream_devox(stream, desc, slot)
        else:
            self.voxel_stream(stream, slot)

    def pipelined_steps(self, steps, batch, consume, select_events=None, prefetch=False,
                        voxel_ahead=False):
        """`steps` train steps whose neighbour side runs one batch ahead.

        A batch's self-KNN + local PPF depend on its coordinates and normals
        only (pvcnn_classify.py:252-269 computes them from the input, before
        any weight), so batch s+1's neighbours run on s_nbr while batch s's
        backward runs on the caller's stream: the VALU-bound selection
        overlaps the HBM-bound voxel passes and backwards.  Per step s, on
        the caller's stream: the voxel side of batch s, a wait for batch s's
        neighbours (the head of the network needs them), then
        consume(s, outputs) -- the rest of the step (the bench: the devox and
        voxelize backwards).  Index sets alternate; batch s+2's neighbours
        wait until step s's consume is done with set s % 2.  batch(s)
        returns (xyz, normals, features) of step s; nothing is skipped:
        every step's neighbours, voxels and consume run once.

        batch(s) may make its tensors on the caller's stream (an H2D copy as
        in train.py:140, an augmentation, the LRF change_coords); s_nbr waits
        for an event recorded on the caller's stream right after it, so a
        batch's neighbours are ordered after its producers.  xyz and normals
        are record_stream'ed to s_nbr, so the caching allocator does not hand
        their blocks out while s_nbr still reads them.

        prefetch=False (the default): batch(s+1) is called after consume(s),
        as the reference's train loop fetches (train.py:138-153): a producer
        may refill the same staging tensors in place and may read weights
        that consume(s) updated.  prefetch=True calls batch(s+1) right after
        step s's neighbours are enqueued, before step s's voxel side and
        consume(s), so batch s+1's neighbours are not ordered after them
        (more overlap; the c3 bench uses it).  It requires batch(s+1) to
        return NEW storage (never a tensor step s still reads) and not to
        depend on consume(s).
        select_events: optional list of (ev0, ev1) per step, recorded on s_nbr
        around that step's selection launch (its in-step duration).
        voxel_ahead=True (needs prefetch=True and the split voxel stage):
        the voxel head of batch s+1 (prep + means, devox) also runs one batch
        ahead, on s_vox, beside step s's grid stream and consume; only the
        grid stream stays on the caller's stream.  The voxel outputs then
        alternate between two sets like the index sets (outputs(slot)); batch
        s+1's head waits until step s-1's consume is done with its set.  The
        second set is this call's only: consume(s, outputs) receives it, and
        after the call outputs(slot) is back to one voxel set.

        (Round 5 changed the default to prefetch=False: callers that relied
        on the overlap pass prefetch=True, as the bench does.)"""
        cur = torch.cuda.current_stream(self.device)
        # set 1's buffers are made here, before s_nbr forks from the caller's
        # stream.  Made lazily inside the loop they could reuse a block the
        # previous step's consume had just freed with its kernels still
        # pending on the caller's stream, and s_nbr wrote them with no order
        # against those kernels (an illegal-address fault on the GPU when the
        # KNN workspace landed there).
        ahead = bool(voxel_ahead) and bool(prefetch) and self._split_voxels()
        self._vsep = ahead
        self._set(1)
        self._ppf(1)
        if ahead:
            self._vset(1)
            self.s_vox.wait_stream(cur)
        self.s_nbr.wait_stream(cur)

        def fetch(s):
            t = batch(s)
            self._check_inputs(*t)
            ev = torch.cuda.Event()
            ev.record(cur)  # after whatever batch(s) enqueued on the caller's stream
            return t, ev

        done = [None, None]

        def head(s, item):
            # batch s's voxel head on s_vox, after its producers and after
            # step s-2's consume (the last reader of set s % 2)
            (hx, _, hf), e_h = item
            q = s & 1
            self.s_vox.wait_event(e_h)
            if done[q] is not None:
                self.s_vox.wait_event(done[q])
            hx.record_stream(self.s_vox)
            hf.record_stream(self.s_vox)
            self.voxel_head(hx, hf, self.s_vox.cuda_stream, q)
            ev = torch.cuda.Event()
            ev.record(self.s_vox)
            return ev

        try:
            nxt = fetch(0) if steps > 0 else None
            e_vh = head(0, nxt) if ahead and steps > 0 else None
            for s in range(steps):
                (xyz, normals, features), e_in = nxt
                q = s & 1
                self.s_nbr.wait_event(e_in)
                xyz.record_stream(self.s_nbr)
                normals.record_stream(self.s_nbr)
                e_nbr = self.enqueue_neighbors(
                    xyz, normals, q, after=done[q],
                    events=select_events[s] if select_events is not None else None)
                if prefetch:
                    # the next batch is produced ahead of this step's voxel side
                    # and consume (its neighbours wait for its producers only)
                    nxt = fetch(s + 1) if s + 1 < steps else None
                if ahead:
                    cur.wait_event(e_vh)
                    self.voxel_tail(cur.cuda_stream, q)
                    e_vh = head(s + 1, nxt) if s + 1 < steps else None
                else:
                    self.enqueue_voxels(xyz, features, cur.cuda_stream, q)
                cur.wait_event(e_nbr)
                consume(s, self.outputs(slot=q, idx_slot=q))
                ev = torch.cuda.Event()
                ev.record(cur)
                done[q] = ev
                if not prefetch:
                    nxt = fetch(s + 1) if s + 1 < steps else None
            cur.wait_stream(self.s_nbr)
            if ahead:
                cur.wait_stream(self.s_vox)
        finally:
            # the second voxel output set serves this call's consume() only:
            # later eager calls (voxel_prep / outputs(slot=1) ...) use set 0
            self._vsep = False

    def outputs(self, slot=0, idx_slot=0):
        _, _, dinds, dwgts, _ = self._set(slot)
        nc, ind, devox, desc = self._vset(slot)
        return {
            "knn_idx": self._set(idx_slot)[4], "local_ppf": self._ppf(idx_slot),
            "norm_coords": nc,
            "ind": ind, "cnt": self.cnt, "grid": self.grid, "devox": devox,
            "dinds": dinds, "dwgts": dwgts, "desc": desc,
        }

    def _get_runner(self, timed_steps):
        """The library runner (its cross-stream events are created once and
        reused by every run); re-made only to grow its timing capacity."""
        if self._runner is not None and self._runner_cap >= timed_steps:
            return self._runner
        self._free_runner()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.load().pcr_runner_create(int(timed_steps), ctypes.byref(h)),
                       "runner_create")
        self._runner, self._runner_cap = h, int(timed_steps)
        return h

    def reserve_timing(self, timed_steps):
        """Create the runner with room for `timed_steps` grid-kernel timing
        pairs now, so a later run_native(..., timed=True) of that many steps
        does not synchronise the device and create events inside a timed
        region."""
        self._get_runner(int(timed_steps))

    def _free_runner(self):
        if getattr(self, "_runner", None) is not None:
            torch.cuda.synchronize(self.device)
            _lib.load().pcr_runner_destroy(self._runner)
        self._runner, self._runner_cap = None, 0

    def __del__(self):
        try:
            self._free_runner()
        except Exception:  # interpreter shutdown
            pass

    def grid_kernel_times(self):
        """Per-step durations (ms) of the grid-stream kernel in the last
        run_native(..., timed=True) call, from HIP events on its stream."""
        if self._runner is None or self._runner_cap == 0:
            return []
        ms = (ctypes.c_float * self._runner_cap)()
        cnt = ctypes.c_int(0)
        _lib.check(_lib.load().pcr_runner_grid_times(self._runner, ms, self._runner_cap,
                                                     ctypes.byref(cnt)), "runner_grid_times")
        return list(ms[:cnt.value])

    def _make_args(self, xyz, normals, features, match):
        """pcr_extractor_args (include/pcr_amd.h) over these inputs and the
        extractor's buffers."""
        s1 = self._set(1)
        a = _lib.ExtractorArgs()
        a.b, a.n, a.c, a.k, a.r, a.relative = self.b, self.n, self.c, self.k, self.r, \
            int(self.relative)
        a.xyz, a.normals, a.features = _ptr(xyz), _ptr(normals), _ptr(features)
        a.knn_idx, a.knn_dist, a.local_ppf = _ptr(self.knn_idx), _ptr(self.knn_dist), \
            _ptr(self.local_ppf)
        a.norm_coords, a.ind, a.cnt, a.grid = _ptr(self.norm_coords), _ptr(self.ind), \
            _ptr(self.cnt), _ptr(self.grid)
        a.devox, a.desc = _ptr(self.devox), _ptr(self.desc)
        a.dinds[0], a.dinds[1] = _ptr(self.dinds), _ptr(s1[2])
        a.dwgts[0], a.dwgts[1] = _ptr(self.dwgts), _ptr(s1[3])
        a.knn_ws[0], a.knn_ws[1] = _ptr(self.knn_ws), _ptr(s1[0])
        a.knn_ws_bytes = self.knn_ws.numel()
        a.vox_ws[0], a.vox_ws[1] = _ptr(self.ws), _ptr(s1[1])
        a.vox_ws_bytes = self.ws.numel()
        if getattr(self, "_ws3", None) is None:
            # the third voxel workspace of runner schedule 7
            self._ws3 = torch.empty_like(self.ws)
            self._order_new_buffers()
        a.vox_ws3 = _ptr(self._ws3)
        a.devox_in_means = 0 if self.stream_devox else 1
        if match is not None:
            if 2 * match.pairs != self.b or match.n != self.n:
                raise RuntimeError("match buffers are for %d pairs of %d points"
                                   % (match.pairs, match.n))
            a.match_pairs = match.pairs
            a.corr12, a.corr21 = _ptr(match.corr12), _ptr(match.corr21)
            a.idx1, a.idx2, a.match_count = _ptr(match.idx1), _ptr(match.idx2), \
                _ptr(match.count)
            a.match_ws, a.match_ws_bytes = _ptr(match.ws), match.ws.numel()
        return a

    def run_native(self, xyz, normals, features, steps, desc_steps=None, schedule=0,
                   timed=False, match=None):
        """`steps` steps over the extractor's single buffer set, enqueued by
        the library's native runner (pcr_extractor_run schedule 0: sort +
        selection + PPF on s_nbr, prep + the fused grid kernel on s_vox).
        One ctypes call for all steps.  The pipelined schedules 6 / 7 need
        distinct output sets per step: run_ring.  timed: only schedules 6 /
        7 bracket grid-stream kernels (grid_kernel_times()).  match: a
        registration.PairMatch whose buffers receive, every step, the
        mutual-NN matching of clouds [0, B/2) against [B/2, B)."""
        self._check_inputs(xyz, normals, features)
        # timed: True = every step, an int N = N steps in the middle of the run
        ntimed = min(steps, (steps if timed is True else int(timed)) if timed else 0)
        runner = self._get_runner(ntimed)
        if self._runner_cap:
            _lib.check(_lib.load().pcr_runner_set_timed(runner, ntimed), "runner_set_timed")
        # the argument block is built once per (inputs, match) and reused:
        # every other pointer is an extractor buffer, fixed for its life
        key = (xyz.data_ptr(), normals.data_ptr(), features.data_ptr(), match)
        if self._args_key != key:
            self._args = self._make_args(xyz, normals, features, match)
            self._args_key = key
        a = self._args
        if desc_steps is not None and tuple(desc_steps.shape) != (steps, self.b, self.c):
            raise RuntimeError("desc_steps must be [steps, B, C]")
        cur = torch.cuda.current_stream(self.device)
        _lib.check(_lib.load().pcr_extractor_run(
            runner, ctypes.byref(a), steps, schedule, _ptr(desc_steps), cur.cuda_stream,
            self.s_nbr.cuda_stream, self.s_pre.cuda_stream, self.s_vox.cuda_stream),
            "extractor_run")
        return self.outputs(slot=0)

    # ------------------------------------------------------------ batch ring
    def ring_outputs(self, nsets, match_pairs=0):
        """The output sets of run_ring: one dict of output tensors per batch
        slot (knn_idx, local_ppf, norm_coords, ind, cnt, grid, devox, desc,
        dinds, dwgts; the matching outputs when match_pairs > 0), made once
        per ring size on the caller's stream."""
        ring = getattr(self, "_ring", None)
        if ring is not None and len(ring) == nsets and self._ring_match == match_pairs:
            return ring
        b, n, c, k, r3 = self.b, self.n, self.c, self.k, self.r ** 3
        e, dev = torch.empty, self.device
        i32, f32 = dict(dtype=torch.int32, device=dev), dict(dtype=torch.float32, device=dev)
        ring = []
        for _ in range(nsets):
            o = {"knn_idx": e((b, k, n), **i32), "local_ppf": e((b, 4, k, n), **f32),
                 "norm_coords": e((b, 3, n), **f32), "ind": e((b, n), **i32),
                 "cnt": e((b, r3), **i32), "grid": e((b, c, r3), **f32),
                 "devox": e((b, c, n), **f32), "desc": e((b, c), **f32),
                 "dinds": e((b, 8, n), **i32), "dwgts": e((b, 8, n), **f32)}
            if self.knn_dist is not None:
                o["knn_dist"] = e((b, k, n), **f32)
            if match_pairs:
                for key in ("corr12", "corr21", "idx1", "idx2"):
                    o[key] = e((match_pairs, n), **i32)
                o["count"] = e((match_pairs,), **i32)
            ring.append(o)
        self._ring, self._ring_match = ring, match_pairs
        self._order_new_buffers()
        return ring

    def run_ring(self, batches, steps, set0=0, desc_steps=None, schedule=6, timed=False,
                 match=None):
        """`steps` pipelined steps of the native runner over a batch ring
        (pcr_extractor_run with nsets = len(batches)): step s reads the
        clouds of batches[(set0 + s) % R] = (xyz, normals, features) and
        writes every output into ring_outputs(R)[(set0 + s) % R], so with
        steps <= R each step's outputs survive the call and are readable on
        the current stream after it.  schedule 6: two voxel
        and two KNN queues, 7: three voxel queues and one KNN queue, 0:
        serial.  timed: bracket the grid-stream kernel of every step (True)
        or of N steps in the middle of the run (an int N) with timing events
        (grid_kernel_times()).  match: a
        registration.PairMatch (its workspace; the matching outputs go to
        the ring sets).  Returns the ring's output sets."""
        if schedule not in (0, 6, 7):
            raise RuntimeError("run_ring needs schedule 0, 6 or 7")
        if schedule >= 6 and len(batches) < schedule - 4:
            raise RuntimeError("run_ring schedule %d needs at least %d batches"
                               % (schedule, schedule - 4))
        R = len(batches)
        if R < 1:
            raise RuntimeError("run_ring needs at least one batch")
        mp = match.pairs if match is not None else 0
        ring = self.ring_outputs(R, mp)
        ntimed = min(steps, (steps if timed is True else int(timed)) if timed else 0)
        runner = self._get_runner(ntimed)
        if self._runner_cap:
            _lib.check(_lib.load().pcr_runner_set_timed(runner, ntimed), "runner_set_timed")
        # the same batch tuples as the last call (tuples are immutable, so
        # the same tensors): checked and keyed then.  Checking 20 batches
        # and keying their pointers cost ~23 us of host time in front of
        # the first launch (scripts/host_enqueue_probe.py)
        prev = self._ring_seen
        if prev is not None and len(prev[0]) == R and prev[1] is match and \
                all(t is u for t, u in zip(batches, prev[0])):
            key = prev[2]
        else:
            for t in batches:
                self._check_inputs(*t)
            key = ("ring", tuple(tuple(x.data_ptr() for x in t) for t in batches), match)
            self._ring_seen = (tuple(batches), match, key)
        if self._args_key != key:
            a = self._make_args(*batches[0], match)
            sets = (_lib.ExtractorSet * R)()
            for i, ((xyz, nrm, feat), o) in enumerate(zip(batches, ring)):
                st = sets[i]
                st.xyz, st.normals, st.features = _ptr(xyz), _ptr(nrm), _ptr(feat)
                for f in ("knn_idx", "local_ppf", "norm_coords", "ind", "cnt", "grid", "devox",
                          "desc", "dinds", "dwgts", "corr12", "corr21", "idx1", "idx2"):
                    setattr(st, f, _ptr(o[f]) if f in o else None)
                st.knn_dist = _ptr(o["knn_dist"]) if "knn_dist" in o else None
                st.match_count = _ptr(o["count"]) if "count" in o else None
            a.nsets, a.sets = R, sets
            self._args, self._args_key, self._ring_sets = a, key, sets
        a = self._args
        a.set0 = int(set0) % R
        if desc_steps is not None and tuple(desc_steps.shape) != (steps, self.b, self.c):
            raise RuntimeError("desc_steps must be [steps, B, C]")
        cur = torch.cuda.current_stream(self.device)
        _lib.check(_lib.load().pcr_extractor_run(
            runner, ctypes.byref(a), steps, schedule, _ptr(desc_steps), cur.cuda_stream,
            self.s_nbr.cuda_stream, self.s_pre.cuda_stream, self.s_vox.cuda_stream),
            "extractor_run")
        return ring

    def capture(self, xyz, normals, features):
        """Capture one step over these input tensors into a hipGraph."""
        self._check_inputs(xyz, normals, features)
        self._static_in = (xyz, normals, features)
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self.forward(xyz, normals, features)  # warm-up outside capture
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cur = self._fork()
            self.enqueue(xyz, normals, features)
            self._join(cur)
        self.graph = g
        return g

    def replay(self):
        self.graph.replay()
        return self.outputs()


def grid_kernel_bytes_per_cloud(n, r, c):
    """Algorithmic HBM bytes of the dominant kernel (vox_grid_kernel<1>: the
    spherical_avg_voxelize output) per cloud: features read
    4CN, grid written 4C r^3, cnt written 4 r^3.  The prep metadata it also
    reads (occupancy bitmap + word prefix r^3/4 bytes, segment offsets and
    point order 8N) is not counted: it is an artefact of this design."""
    r3 = r ** 3
    return 4 * c * n + 4 * c * r3 + 4 * r3


def stream_kernel_bytes_per_cloud(r, c, n=None):
    """Algorithmic HBM bytes of the split voxel stage's dominant kernel
    (vox_stream_kernel: the spherical_avg_voxelize outputs)
    per cloud: grid written 4C r^3, cnt written 4 r^3; with n (the kernel's
    devox role, clouds of <= 1024 points) also the spherical devox of 8d:
    devox written 4CN, the corner data read 64N, the descriptor written 4C.
    Its reads of the compact voxel means (4C per occupied voxel) and of the
    occupancy bitmap are artefacts of this design and not counted."""
    r3 = r ** 3
    b = 4 * c * r3 + 4 * r3
    if n is not None:
        b += 4 * c * n + 64 * n + 4 * c
    return b


def fused_grid_kernel_bytes_per_cloud(n, r, c):
    """Algorithmic HBM bytes of the step's voxel kernel (vox_grid_kernel<3>:
    spherical_avg_voxelize output + spherical_trilinear_devoxelize of it +
    descriptor) per cloud: features read 4CN, grid written
    4C r^3, cnt 4 r^3, devox written 4CN, corner inds + wgts read 64N,
    descriptor 4C.  Prep's corner -> segment map (32N) and the occupancy
    metadata are artefacts of this design and not counted."""
    return grid_kernel_bytes_per_cloud(n, r, c) + 4 * c * n + 64 * n + 4 * c


def algorithmic_bytes_per_cloud(n, k, r, c):
    """SURVEY.md 8d per-cloud byte model (the roofline.achieved numerator):
    KNN 12N + 4kN; local PPF 24N + 16kN; sph-vox 12N + 4CN + 4N + 4r^3 + 4C r^3;
    sph-devox 12N + 4N + 320C + 4CN + 64N."""
    r3 = r ** 3
    knn = 12 * n + 4 * k * n
    lppf = 24 * n + 16 * k * n
    vox = 12 * n + 4 * c * n + 4 * n + 4 * r3 + 4 * c * r3
    devox = 12 * n + 4 * n + 4 * 80 * c + 4 * c * n + 64 * n
    return {"knn": knn, "local_ppf": lppf, "sph_vox": vox, "sph_devox": devox,
            "total": knn + lppf + vox + devox}
