"""CPU: the oracle restatements of SURVEY.md 8f rows f2 (LRF change_coords,
models/pvcnn_classify.py:153-184) and f4 (PointNet++ ops, sampling.cu,
neighbor_interpolate.cu), checked against independent PyTorch/NumPy
restatements of the reference's code.  The reference itself cannot run here
(SURVEY.md 8c), so these pins are "parity unpinned" against genuine reference
output.  The oracle is the checker of the GPU tests
(tests/test_gpu_pointnet2_lrf.py)."""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds


def torch_change_coords(coords):
    """The reference's change_coords block, restated on CPU torch fp32, with
    a stable argsort (the reference's argsort leaves ties open)."""
    x = torch.from_numpy(coords)
    b, _, n = x.shape
    nc = x - x.mean(dim=2, keepdim=True)
    rank = torch.argsort(nc.norm(dim=1), dim=1, descending=True, stable=True)
    bx_all = torch.zeros(b, 3, 1)
    by_all = torch.zeros(b, 3, 1)
    picks = []
    for i in range(b):
        bx = nc[i, :, rank[i, 0]]
        assert bx.norm() > 1e-5
        bx = bx / bx.norm()
        pick = None
        for j in range(1, n):
            by = nc[i, :, rank[i, j]]
            if by.norm() < 1e-5:
                continue
            by = by / by.norm()
            lam = (bx * by).sum()
            if -0.9 < lam < 0.9:
                pick = int(rank[i, j])
                break
        assert pick is not None
        picks.append((int(rank[i, 0]), pick))
        bx_all[i, :, 0] = bx
        by_all[i, :, 0] = by
    bx_all -= by_all * bx_all.permute(0, 2, 1).bmm(by_all)
    bx_all /= bx_all.norm(dim=1, keepdim=True)
    bz = torch.cross(bx_all, by_all, dim=1)
    bz = bz / bz.norm(dim=1, keepdim=True)
    out = torch.cat([v.permute(0, 2, 1).bmm(nc) for v in (bx_all, by_all, bz)], dim=1)
    return out.numpy(), np.array(picks, np.int32)


@pytest.mark.parametrize("b,n", [(3, 1024), (2, 37), (1, 2048)])
def test_oracle_lrf_matches_torch_restatement(b, n):
    xyz, _, _ = gaussian_clouds(b, n, seed=n)
    xyz = xyz + np.float32(0.25)  # non-centred input: the block centres it
    out, basis, picks, status = oracle.lrf_change_coords(xyz)
    ref, ref_picks = torch_change_coords(xyz)
    assert (status == 0).all()
    assert np.array_equal(picks, ref_picks)
    assert np.abs(out - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    for q in range(b):  # orthonormal, right-handed
        assert np.allclose(basis[q] @ basis[q].T, np.eye(3), atol=1e-6)
        assert np.linalg.det(basis[q]) > 0.999


def test_oracle_lrf_rotation_invariance():
    """The frame turns with the cloud: new coords of R x equal those of x."""
    xyz, _, _ = gaussian_clouds(2, 700, seed=3)
    rng = np.random.default_rng(0)
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    if np.linalg.det(q) < 0:
        q[:, 0] = -q[:, 0]
    rot = np.einsum("ij,bjn->bin", q, xyz.astype(np.float64)).astype(np.float32)
    a, _, pa, _ = oracle.lrf_change_coords(xyz)
    r, _, pr, _ = oracle.lrf_change_coords(rot)
    assert np.array_equal(pa, pr)
    assert np.abs(a - r).max() < 1e-4


def test_oracle_lrf_asserts():
    # all points at the centroid: base_x has norm 0 (:159)
    z = np.zeros((1, 3, 16), np.float32)
    assert oracle.lrf_change_coords(z)[3][0] == 1
    # collinear cloud: no base_y with |lambda| < 0.9 (:169)
    t = np.linspace(-1, 1, 33, dtype=np.float32)
    line = np.stack([t, 2 * t, -t])[None]
    assert oracle.lrf_change_coords(line)[3][0] == 2


def test_oracle_fps_ties_follow_the_512_thread_reduction():
    """Every point at the same distance: the reference's reduction picks the
    lowest thread (k % 512) first, not the lowest index."""
    n = 1100
    # integer lattice points: every squared distance is exact, ties abound
    g = np.arange(n)
    xyz = np.stack([g % 11, (g // 11) % 10, g // 110]).astype(np.float32)[None]
    xyz[:, :, 512:] = xyz[:, :, :n - 512]  # k and k+512 coincide
    idx = oracle.furthest_point_sampling(xyz, 12)
    assert idx[0, 0] == 0
    # a brute-force restatement with the same thread structure
    X = xyz[0]
    dist = np.full(n, 1e38, np.float32)
    old, exp = 0, [0]
    for _ in range(11):
        d = ((X[0] - X[0, old]) ** 2 + (X[1] - X[1, old]) ** 2 + (X[2] - X[2, old]) ** 2)
        dist = np.minimum(dist, d.astype(np.float32))
        best = dist.max()
        cand = np.nonzero(dist == best)[0]
        old = int(min(cand, key=lambda k: (k % 512, k)))
        exp.append(old)
    assert idx[0].tolist() == exp


def test_oracle_fps_matches_numpy_on_generic_clouds():
    xyz, _, _ = gaussian_clouds(2, 900, seed=7)
    idx = oracle.furthest_point_sampling(xyz, 64)
    for q in range(2):
        X = xyz[q].astype(np.float64)
        dist = np.full(900, np.inf)
        old, exp = 0, [0]
        for _ in range(63):
            dist = np.minimum(dist, ((X - X[:, old:old + 1]) ** 2).sum(0))
            old = int(np.argmax(dist))
            exp.append(old)
        assert idx[q].tolist() == exp


def test_oracle_three_nn_matches_numpy():
    rng = np.random.default_rng(2)
    b, n, m, c = 2, 300, 77, 5
    pts = rng.standard_normal((b, 3, n)).astype(np.float32)
    ctr = rng.standard_normal((b, 3, m)).astype(np.float32)
    cf = rng.standard_normal((b, c, m)).astype(np.float32)
    out, inds, wgts = oracle.three_nearest_neighbors_interpolate_forward(pts, ctr, cf)
    for q in range(b):
        d = ((pts[q][:, :, None].astype(np.float64) - ctr[q][:, None, :]) ** 2).sum(0)
        order = np.argsort(d, axis=1, kind="stable")[:, :3]
        assert np.array_equal(inds[q].T, order)
        dd = np.maximum(np.take_along_axis(d, order, 1), 1e-10)
        w = (1.0 / dd) / (1.0 / dd).sum(1, keepdims=True)
        assert np.abs(wgts[q].T - w).max() < 1e-5
        ref = np.einsum("cnk,nk->cn", cf[q][:, order], w)
        assert np.abs(out[q] - ref).max() < 1e-5
    g = rng.standard_normal((b, c, n)).astype(np.float32)
    gx = oracle.three_nearest_neighbors_interpolate_backward(g, inds, wgts, m)
    exp = np.zeros((b, c, m))
    for q in range(b):
        for a in range(3):
            np.add.at(exp[q].T, inds[q, a], (g[q] * wgts[q, a]).T)
    assert np.abs(gx - exp).max() < 1e-5


def test_oracle_three_nn_fewer_than_three_centres():
    pts = np.zeros((1, 3, 4), np.float32)
    ctr = np.ones((1, 3, 2), np.float32)
    cf = np.array([[[1.0, 3.0]]], np.float32)
    out, inds, wgts = oracle.three_nearest_neighbors_interpolate_forward(pts, ctr, cf)
    assert inds[0, :, 0].tolist() == [0, 1, 0]  # unfilled slot keeps index 0
    assert abs(wgts[0, 2, 0]) < 1e-9          # 1e10 clamp -> negligible weight


def test_oracle_gather_roundtrip():
    rng = np.random.default_rng(4)
    f = rng.standard_normal((2, 4, 50)).astype(np.float32)
    idx = rng.integers(0, 50, (2, 30)).astype(np.int32)
    out = oracle.gather_features_forward(f, idx)
    assert np.array_equal(out, np.take_along_axis(f, idx[:, None, :].repeat(4, 1), 2))
    g = rng.standard_normal((2, 4, 30)).astype(np.float32)
    gx = oracle.gather_features_backward(g, idx, 50)
    exp = np.zeros((2, 4, 50), np.float32)
    for q in range(2):
        np.add.at(exp[q].T, idx[q], g[q].T)
    assert np.abs(gx - exp).max() < 1e-5


def test_losses_match_reference_formulas():
    import PVCNN.modules.functional as F
    torch.manual_seed(0)
    x, y = torch.randn(4, 6), torch.randn(4, 6)
    p = torch.softmax(x, 1)
    exp = torch.mean(torch.sum(p * (torch.log(p) - torch.log_softmax(y, 1)), 1))
    assert torch.allclose(F.kl_loss(x, y), exp)
    e = torch.randn(100) * 3
    q = torch.minimum(e.abs(), torch.full_like(e, 1.5))
    assert torch.allclose(F.huber_loss(e, 1.5), torch.mean(0.5 * q ** 2 + 1.5 * (e.abs() - q)))
