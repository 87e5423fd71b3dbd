"""Fused sph-dg extractor forward: the north-star hot path as one step.

One step over a batch of clouds (xyz [B,3,N], normals [B,3,N], point
features [B,C,N], all resident on the GPU):

  neighbour stage (stream A): self-KNN (k) -> local PPF [B,4,k,N]
      = knn_forward_cuda + the model's local-PPF block
        (PVCNN/models/pvcnn_classify.py:252-269), fused in one kernel
  voxel stage (stream B): Spherical_Voxelization normalisation
      (PVCNN/modules/spherical_vox.py:16-20) + voxel index / occupancy (prep),
      then spherical_avg_voxelize's dense grid [B,C,r^3] + cnt (grid kernel),
      and on stream C the spherical_trilinear_devoxelize of that grid
      ([B,C,N] + inds/wgts) + per-cloud descriptor (max over points) [B,C]
      (devox kernel; it re-forms the voxel means in LDS instead of re-reading
      the grid, so it runs beside the grid kernel)

The stages run on HIP streams forked from and joined back to the caller's
stream.  ``capture()`` records one step into a hipGraph; ``run_pipelined()``
enqueues S consecutive steps with no join between them, so step i+1's
neighbour stage overlaps step i's voxel stage.
"""
import torch

from . import _lib
from .ops import _ptr


class SphExtractor:
    def __init__(self, batch, npoints, channels, k, resolution, device="cuda", relative=True,
                 with_dist=False):
        self.b, self.n, self.c, self.k, self.r = batch, npoints, channels, k, resolution
        self.relative = relative
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
        self.s_nbr = torch.cuda.Stream(device=dev)
        self.s_vox = torch.cuda.Stream(device=dev)
        self.s_dev = torch.cuda.Stream(device=dev)
        self.graph = None
        self._static_in = None

    # ---------------------------------------------------------------- stages
    def neighbor_stage(self, xyz, normals, stream):
        _lib.check(_lib.load().pcr_knn_local_ppf(
            _ptr(xyz), _ptr(normals), self.b, self.n, self.k, int(self.relative),
            _ptr(self.knn_idx), _ptr(self.knn_dist), _ptr(self.local_ppf), _ptr(self.knn_ws),
            self.knn_ws.numel(), stream), "knn_local_ppf")

    def voxel_stage(self, xyz, features, stream):
        _lib.check(_lib.load().pcr_extractor_voxel_stage(
            _ptr(xyz), _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.norm_coords),
            _ptr(self.ind), _ptr(self.cnt), _ptr(self.grid), _ptr(self.devox), _ptr(self.dinds),
            _ptr(self.dwgts), _ptr(self.desc), _ptr(self.ws), self.ws.numel(), stream),
            "extractor_voxel_stage")

    def voxel_prep(self, xyz, stream):
        _lib.check(_lib.load().pcr_extractor_voxel_prep(
            _ptr(xyz), self.b, self.n, self.r, _ptr(self.norm_coords), _ptr(self.ind),
            _ptr(self.dinds), _ptr(self.dwgts), _ptr(self.ws), self.ws.numel(), stream),
            "extractor_voxel_prep")

    def voxel_grid(self, features, stream):
        """The dominant kernel (vox_grid_kernel<1>: means -> dense grid + cnt)."""
        _lib.check(_lib.load().pcr_extractor_voxel_grid(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.cnt), _ptr(self.grid),
            _ptr(self.ws), self.ws.numel(), stream), "extractor_voxel_grid")

    def voxel_devox(self, features, stream, desc=None):
        d = self.desc if desc is None else desc
        _lib.check(_lib.load().pcr_extractor_voxel_devox(
            _ptr(features), self.b, self.c, self.n, self.r, _ptr(self.devox), _ptr(self.dinds),
            _ptr(self.dwgts), _ptr(d), _ptr(self.ws), self.ws.numel(), stream),
            "extractor_voxel_devox")

    def _check_inputs(self, xyz, normals, features):
        for t, name in ((xyz, "xyz"), (normals, "normals"), (features, "features")):
            if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
                raise RuntimeError("%s must be a contiguous float CUDA tensor" % name)
        if tuple(xyz.shape) != (self.b, 3, self.n) or tuple(features.shape) != (self.b, self.c,
                                                                                  self.n):
            raise RuntimeError("input shape does not match the extractor configuration")

    def enqueue(self, xyz, normals, features, desc=None, first=True):
        """Enqueue one step on the extractor's own streams, no fork/join.
        Stream order carries the step-to-step dependencies, so consecutive
        steps pipeline: step i+1's neighbour stage runs beside step i's voxel
        stage.  The only cross-stream edges: devox after prep (it reads the
        prep results) and the next prep after devox (prep overwrites them);
        `first` = nothing of this extractor is pending on the streams since
        the last fork (no previous devox to wait for)."""
        self.neighbor_stage(xyz, normals, self.s_nbr.cuda_stream)
        if not first:
            self.s_vox.wait_stream(self.s_dev)
        self.voxel_prep(xyz, self.s_vox.cuda_stream)
        self.s_dev.wait_stream(self.s_vox)
        self.voxel_grid(features, self.s_vox.cuda_stream)
        self.voxel_devox(features, self.s_dev.cuda_stream, desc)

    def _fork(self):
        cur = torch.cuda.current_stream(self.device)
        for st in (self.s_nbr, self.s_vox, self.s_dev):
            st.wait_stream(cur)
        return cur

    def _join(self, cur):
        for st in (self.s_nbr, self.s_vox, self.s_dev):
            cur.wait_stream(st)

    def forward(self, xyz, normals, features):
        """Enqueue one step, forked from and joined back to the current stream."""
        self._check_inputs(xyz, normals, features)
        cur = self._fork()
        self.enqueue(xyz, normals, features)
        self._join(cur)
        return self.outputs()

    def outputs(self):
        return {
            "knn_idx": self.knn_idx, "local_ppf": self.local_ppf, "norm_coords": self.norm_coords,
            "ind": self.ind, "cnt": self.cnt, "grid": self.grid, "devox": self.devox,
            "dinds": self.dinds, "dwgts": self.dwgts, "desc": self.desc,
        }

    def run_pipelined(self, xyz, normals, features, steps, desc_steps=None):
        """Enqueue `steps` consecutive steps with no join between them (step
        i+1's neighbour stage overlaps step i's voxel stage), forked from and
        joined back to the current stream once.  Step s writes its descriptor
        to desc_steps[s] when given.  Eager launches: ROCm's stream capture
        does not take the prep-after-devox edge between two steps."""
        self._check_inputs(xyz, normals, features)
        cur = self._fork()
        for s in range(steps):
            d = None if desc_steps is None else desc_steps[s]
            self.enqueue(xyz, normals, features, desc=d, first=s == 0)
        self._join(cur)
        return self.outputs()

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
