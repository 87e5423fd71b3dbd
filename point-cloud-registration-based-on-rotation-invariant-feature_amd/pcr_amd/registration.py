"""Registration pairs on one rank (BASELINE c4).

The reference's registration evaluation extracts per-point features of the
source and the target cloud of every pair (datasets/deepgmr_mn40.py:71-97:
feat1 = model(pc1), feat2 = model(pc2)) and matches them by mutual nearest
neighbours in feature space (:232-244, find_correspondence_one_pair).  Here
one step of a rank's shard of P pairs is:

  * the extractor forward (pcr_amd.extractor.SphExtractor, the north-star
    hot path) over a batch of 2P clouds -- sources in [0, P), targets in
    [P, 2P) -- so both clouds of a pair live on the same rank;
  * the mutual-NN matching of each source's devoxelised per-point features
    [C, N] against its target's (pcr_mutual_nn_match_cm, fp32 MFMA), which
    needs no exchange because the pair is local;
  * the per-cloud descriptors [2P, C] of the step, all-gathered across ranks
    (pcr_amd.distributed.gather_descriptors, RCCL over xGMI) -- the only
    collective.

The native runner (pcr_extractor_run with match_pairs = P) enqueues the
matching on each step's voxel queue right after its devox (behind the grid
stream, which evaluates the devox at c2-sized clouds), so S steps of
extraction + matching cost one host call.
"""
import torch

from . import _lib, ops
from .extractor import SphExtractor


class PairMatch:
    """Output and workspace buffers of the per-step matching of P pairs of
    N-point clouds: corr12 / corr21 / idx1 / idx2 [P, N] int32, count [P]."""

    def __init__(self, pairs, npoints, device):
        self.pairs, self.n = int(pairs), int(npoints)
        i32 = dict(dtype=torch.int32, device=device)
        self.corr12 = torch.empty((pairs, npoints), **i32)
        self.corr21 = torch.empty((pairs, npoints), **i32)
        self.idx1 = torch.empty((pairs, npoints), **i32)
        self.idx2 = torch.empty((pairs, npoints), **i32)
        self.count = torch.empty((pairs,), **i32)
        need = _lib.load().pcr_mutual_nn_workspace_size(pairs, npoints, npoints)
        # three parts: the runner's schedules 6 / 7 match consecutive steps
        # on two / three queues at once, each in its own part
        part = (max(256, need) + 255) // 256 * 256
        self.ws = torch.empty(3 * part + 768, dtype=torch.uint8, device=device)

    def outputs(self):
        return {"corr12": self.corr12, "corr21": self.corr21, "idx1": self.idx1,
                "idx2": self.idx2, "count": self.count}


class PairExtractor:
    """Extraction + matching of a rank's P registration pairs per step."""

    def __init__(self, pairs, npoints, channels, k, resolution, device="cuda", relative=True):
        self.pairs = int(pairs)
        self.ex = SphExtractor(2 * pairs, npoints, channels, k, resolution, device=device,
                               relative=relative)
        self.match = PairMatch(pairs, npoints, self.ex.device)

    @staticmethod
    def pack(src, tgt):
        """[P, ...] sources and targets -> the [2P, ...] batch of one step."""
        return torch.cat((src, tgt), dim=0).contiguous()

    def forward(self, xyz, normals, features):
        """One step from Python: extractor forward, then the matching on the
        current stream.  Inputs are the packed [2P, ...] batch."""
        out = dict(self.ex.forward(xyz, normals, features))
        p = self.pairs
        dv = out["devox"]
        got = ops.mutual_nn_match(dv[:p], dv[p:], channel_major=True, workspace=self.match.ws)
        out.update(zip(("corr12", "corr21", "idx1", "idx2", "count"), got))
        return out

    def run_native(self, xyz, normals, features, steps, desc_steps=None, schedule=0,
                   timed=False):
        """`steps` serial steps of extraction + matching from one native
        runner call (schedule 0); the matching outputs of the last step stay
        in self.match."""
        out = dict(self.ex.run_native(xyz, normals, features, steps, desc_steps,
                                      schedule=schedule, timed=timed, match=self.match))
        out.update(self.match.outputs())
        return out

    def run_ring(self, batches, steps, set0=0, desc_steps=None, schedule=6, timed=False):
        """`steps` pipelined steps of extraction + matching over a batch ring
        of packed [2P, ...] batches (SphExtractor.run_ring): step s matches
        the pairs of batches[(set0 + s) % R] into that ring set's corr12 /
        corr21 / idx1 / idx2 / count."""
        return self.ex.run_ring(batches, steps, set0, desc_steps, schedule=schedule,
                                timed=timed, match=self.match)

    def grid_kernel_times(self):
        return self.ex.grid_kernel_times()

    def reserve_timing(self, timed_steps):
        self.ex.reserve_timing(timed_steps)
