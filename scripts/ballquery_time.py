"""Times the sph-dg model's neighbour path (pvcnn_classify.py:252-271) at
BASELINE c2 (32 x 1024 points): BallQuery(r=0.3, u=128) + local PPF
[B,4,128,N], as the fused two-kernel path (pcr_ball_query +
pcr_local_ppf_forward) and as the reference's composition (BallQuery's two
grouping launches + ~10 torch kernels) on the same ball-query kernel; HIP
events on the current stream.  usage: python scripts/ballquery_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import PVCNN.modules.functional as F  # noqa: E402
from PVCNN.modules.ball_query import BallQuery  # noqa: E402
from pcr_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return t[len(t) // 2] * 1e3


def composition(coords, normals, grouper, u):
    g = grouper(coords, coords, normals)
    nbr_c, nbr_n = g[:, :3], g[:, 3:]
    cc = coords.unsqueeze(2).expand(-1, -1, u, -1)
    cn = normals.unsqueeze(2).expand(-1, -1, u, -1)
    d = cc - nbr_c
    dn = torch.norm(d, dim=1, p=2, keepdim=True)
    du = d / dn
    nr_d = torch.acos(nbr_n.mul(du).sum(dim=1, keepdim=True).clamp(-1, 1))
    ni_d = torch.acos(cn.mul(du).sum(dim=1, keepdim=True).clamp(-1, 1))
    nr_ni = torch.acos(nbr_n.mul(cn).sum(dim=1, keepdim=True).clamp(-1, 1))
    return torch.cat((nr_d, ni_d, nr_ni, dn), dim=1)


for b, n in ((32, 1024), (32, 2048)):
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev) * 0.35
    xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
    nrm = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
    r, u = 0.3, 128
    idx = F.ball_query(xyz, xyz, r, u)
    filled = float((idx != idx[:, :, :1]).float().sum(2).add(1).mean())
    t_bq = timed(lambda: F.ball_query(xyz, xyz, r, u))
    t_ppf = timed(lambda: F.local_ppf(xyz, nrm, idx))
    t_fused = timed(lambda: F.local_ppf(xyz, nrm, F.ball_query(xyz, xyz, r, u)))
    grouper = BallQuery(r, u, include_coordinates=True)
    t_comp = timed(lambda: composition(xyz, nrm, grouper, u))
    out_bytes = b * 4 * u * n * 4
    print("b=%d n=%d r=%.1f u=%d (~%.0f distinct neighbours per centre): ball_query %.1f us, "
          "local_ppf %.1f us (%.0f GB/s of output), fused path %.1f us, reference "
          "composition %.1f us" % (b, n, r, u, filled, t_bq, t_ppf, out_bytes / t_ppf / 1e3,
                                   t_fused, t_comp), flush=True)
