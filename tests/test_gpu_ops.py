"""GPU parity: every hot-path op through the C ABI vs the golden fixtures and the
CPU oracle.  Indices must match bit for bit; floats within the north-star
tolerance (1e-5 abs) -- most are in fact bit-identical because the kernels
and the oracle share include/pcr_math.h and the same accumulation order."""
import os

import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds, edge_norm_coords
from sumorder import (assert_within_sum_order, devox_backward_bound, grouping_backward_bound,
                      knn_backward_bound)

pytestmark = pytest.mark.gpu

GOLDEN = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
TOL = 1e-5  # north_star: PPF angles and devoxelised features within 1e-5 fp32


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def close(a, b, tol=TOL, rtol=0.0):
    """|a - b| <= tol + rtol |b| elementwise, NaN where both are NaN."""
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    both_nan = np.isnan(a) & np.isnan(b)
    diff = np.abs(np.where(both_nan, 0, a - b))
    assert not np.isnan(diff).any(), "NaN mismatch"
    excess = diff - (tol + rtol * np.abs(np.where(both_nan, 0, b)))
    assert excess.max(initial=0) <= 0, diff.max()


# scatter-add backward passes sum in atomic (arbitrary) order, as the
# reference's do: fp32 sum-order tolerance 1e-4 absolute + 1e-5 relative
SCATTER_RTOL = 1e-5


# --------------------------------------------------------------- voxelize
def test_sph_vox_golden(dev):
    from pcr_amd import ops
    g = GOLDEN
    out, ind, cnt = ops.spherical_avg_voxelize_forward(T(g["svox_feat"], dev),
                                                       T(g["svox_coords"], dev), int(g["svox_r"]))
    assert np.array_equal(N(ind), g["svox_ind"])
    assert np.array_equal(N(cnt), g["svox_cnt"])
    assert np.array_equal(N(out), g["svox_out"])  # same summation order -> bit-exact
    assert N(ind)[0, 0] == 2056


@pytest.mark.parametrize("b,n,c,r", [(1, 1024, 64, 16), (32, 1024, 64, 32), (3, 2048, 67, 32),
                                     (2, 777, 5, 7), (2, 4096, 3, 64)])
def test_sph_vox_random(dev, b, n, c, r):
    from pcr_amd import ops
    xyz, _, feat = gaussian_clouds(b, n, seed=b * 7 + n, c=c)
    nc = oracle.normalize_sph(xyz)
    out, ind, cnt = ops.spherical_avg_voxelize_forward(T(feat, dev), T(nc, dev), r)
    eo, ei, ec = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    assert np.array_equal(N(ind), ei)
    assert np.array_equal(N(cnt), ec)
    assert np.array_equal(N(out), eo)


def test_sph_vox_backward(dev):
    from pcr_amd import ops
    g = GOLDEN
    gx = ops.spherical_avg_voxelize_backward(T(g["svox_grad_y"], dev), T(g["svox_ind"], dev),
                                             T(g["svox_cnt"], dev))
    assert np.array_equal(N(gx), g["svox_grad_x"])


def test_cube_vox_golden(dev):
    from pcr_amd import ops
    g = GOLDEN
    out, ind, cnt = ops.avg_voxelize_forward(T(g["cvox_feat"], dev), T(g["cvox_vc"], dev),
                                             int(g["cvox_r"]))
    assert np.array_equal(N(ind), g["cvox_ind"])
    assert np.array_equal(N(cnt), g["cvox_cnt"])
    assert np.array_equal(N(out), g["cvox_out"])


def test_normalize(dev):
    from pcr_amd import ops
    out = ops.spherical_normalize(T(GOLDEN["norm_in"], dev))
    assert np.array_equal(N(out), GOLDEN["norm_out"])


# ------------------------------------------------------------- devoxelize
def test_sph_devox_golden(dev):
    from pcr_amd import ops
    g = GOLDEN
    r = int(g["svox_r"])
    outs, inds, wgts = ops.spherical_trilinear_devoxelize_forward(
        r, True, T(g["svox_coords"], dev), T(g["sdevox_grid"], dev), T(g["svox_ind"], dev))
    assert np.array_equal(N(inds), g["sdevox_inds"])
    assert np.array_equal(N(wgts), g["sdevox_wgts"])
    close(N(outs), g["sdevox_outs"])
    assert np.array_equal(N(outs), g["sdevox_outs"])


def test_sph_devox_backward(dev):
    from pcr_amd import ops
    g = GOLDEN
    r = int(g["svox_r"])
    gx = ops.spherical_trilinear_devoxelize_backward(
        T(g["sdevox_grad_y"], dev), T(g["sdevox_inds"], dev), T(g["sdevox_wgts"], dev), r)
    bound = devox_backward_bound(g["sdevox_grad_y"], g["sdevox_inds"], g["sdevox_wgts"], r ** 3,
                                 skip_neg=True)
    assert_within_sum_order(N(gx), g["sdevox_grad_x"], bound)


def test_cube_devox_golden(dev):
    from pcr_amd import ops
    g = GOLDEN
    rc = int(g["cvox_r"])
    outs, inds, wgts = ops.trilinear_devoxelize_forward(rc, True, T(g["cvox_cc"], dev),
                                                        T(g["cdevox_grid"], dev))
    assert np.array_equal(N(inds), g["cdevox_inds"])
    assert np.array_equal(N(wgts), g["cdevox_wgts"])
    close(N(outs), g["cdevox_outs"])
    gx = ops.trilinear_devoxelize_backward(T(g["cdevox_grad_y"], dev), inds, wgts, rc)
    bound = devox_backward_bound(g["cdevox_grad_y"], g["cdevox_inds"], g["cdevox_wgts"], rc ** 3)
    assert_within_sum_order(N(gx), g["cdevox_grad_x"], bound)


@pytest.mark.parametrize("b,n,c,r", [(4, 1024, 64, 32), (2, 2048, 16, 16)])
def test_sph_devox_random(dev, b, n, c, r):
    from pcr_amd import ops
    xyz, _, feat = gaussian_clouds(b, n, seed=5, c=c)
    nc = oracle.normalize_sph(xyz)
    _, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    grid = np.random.default_rng(9).standard_normal((b, c, r ** 3)).astype(np.float32)
    outs, inds, wgts = ops.spherical_trilinear_devoxelize_forward(r, False, T(nc, dev),
                                                                  T(grid, dev), T(ind, dev))
    eo, ei, ew = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    assert np.array_equal(N(outs), eo)
    gy = np.random.default_rng(3).standard_normal((b, c, n)).astype(np.float32)
    gx = ops.spherical_trilinear_devoxelize_backward(T(gy, dev), inds, wgts, r)
    assert_within_sum_order(N(gx), oracle.devoxelize_backward(gy, ei, ew, r, spherical=True),
                            devox_backward_bound(gy, ei, ew, r ** 3, skip_neg=True))


# -------------------------------------------------------------------- KNN
def test_knn_golden(dev):
    from pcr_amd import ops
    g = GOLDEN
    d1, d2, i1, i2 = ops.knn_forward_cuda(T(g["knn_x1"], dev), T(g["knn_x2"], dev),
                                          int(g["knn_k"]))
    assert np.array_equal(N(i1), g["knn_i1"])
    assert np.array_equal(N(i2), g["knn_i2"])
    assert np.array_equal(N(d1), g["knn_d1"])
    assert np.array_equal(N(d2), g["knn_d2"])


def test_knn_unfilled_slots(dev):
    from pcr_amd import ops
    g = GOLDEN
    xs = g["knn_small_x"]
    d1, d2, i1, i2 = ops.knn_forward_cuda(T(xs, dev), T(xs[:, :, :7], dev), 12)
    assert np.array_equal(N(d1), g["knn_small_d1"]) and np.array_equal(N(i1), g["knn_small_i1"])
    assert np.array_equal(N(d2), g["knn_small_d2"]) and np.array_equal(N(i2), g["knn_small_i2"])


@pytest.mark.parametrize("b,n,m,k", [(2, 1024, 1024, 32), (1, 1000, 513, 16), (1, 300, 300, 64),
                                     (1, 200, 220, 100), (1, 64, 70, 130)])
def test_knn_random(dev, b, n, m, k):
    from pcr_amd import ops
    rng = np.random.default_rng(n + k)
    x1 = rng.standard_normal((b, 3, n)).astype(np.float32)
    x2 = rng.standard_normal((b, 3, m)).astype(np.float32)
    d1, d2, i1, i2 = ops.knn_forward_cuda(T(x1, dev), T(x2, dev), k)
    e = oracle.knn_forward(x1, x2, k)
    for got, exp in zip((d1, d2, i1, i2), e):
        assert np.array_equal(N(got), exp)


def test_knn_general_c(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(1)
    x1 = rng.standard_normal((2, 5, 300)).astype(np.float32)
    x2 = rng.standard_normal((2, 5, 250)).astype(np.float32)
    got = ops.knn_forward_cuda(T(x1, dev), T(x2, dev), 20)
    for a, b in zip(got, oracle.knn_forward(x1, x2, 20)):
        assert np.array_equal(N(a), b)


def test_knn_backward(dev):
    from pcr_amd import ops
    g = GOLDEN
    g1, g2 = ops.knn_backward_cuda(T(g["knn_x1"], dev), T(g["knn_x2"], dev), T(g["knn_gd1"], dev),
                                   T(g["knn_gd2"], dev), T(g["knn_i1"], dev), T(g["knn_i2"], dev))
    b1, b2 = knn_backward_bound(g["knn_x1"], g["knn_x2"], g["knn_gd1"], g["knn_gd2"],
                                g["knn_i1"], g["knn_i2"])
    assert_within_sum_order(N(g1), g["knn_g1"], b1)
    assert_within_sum_order(N(g2), g["knn_g2"], b2)


@pytest.mark.parametrize("self_knn", [True, False])
def test_knn_backward_c2_shape(dev, self_knn):
    """knn_backward_cuda at the c2 shape (B=4, N=M=1024, k=32) against the
    oracle (ascending order) under the per-element sum-order bound; some
    gradients at the reference's skip value (2 gd >= 20000, knn.cu:68)."""
    from pcr_amd import ops
    b, n, k = 4, 1024, 32
    x1, _, _ = gaussian_clouds(b, n, seed=21)
    x2 = x1 if self_knn else gaussian_clouds(b, n, seed=22)[0]
    _, _, i1, i2 = oracle.knn_forward(x1, x2, k)
    rng = np.random.default_rng(23)
    gd1 = rng.standard_normal((b, k, n)).astype(np.float32)
    gd2 = rng.standard_normal((b, k, n)).astype(np.float32)
    gd1[:, -1, ::7] = 10000.0
    gd2[:, 0, ::5] = 10000.0
    g1, g2 = ops.knn_backward_cuda(T(x1, dev), T(x2, dev), T(gd1, dev), T(gd2, dev),
                                   T(i1, dev), T(i2, dev))
    e1, e2 = oracle.knn_backward(x1, x2, gd1, gd2, i1, i2)
    b1, b2 = knn_backward_bound(x1, x2, gd1, gd2, i1, i2)
    assert_within_sum_order(N(g1), e1, b1)
    assert_within_sum_order(N(g2), e2, b2)


def test_knn_backward_hub_neighbour(dev):
    """A hub neighbour: point 0 is the first neighbour of every point of
    both clouds (8,192 points, k = 8), so its pair list holds 8,192 pairs.
    The stable radix sort by target orders it in O(P) (the old rank scan
    read the whole segment per pair: 6.7e7 reads).  Within the sum-order
    bound of the oracle, bit-repeatable, time printed."""
    from pcr_amd import ops
    b, n, k = 2, 8192, 8
    rng = np.random.default_rng(27)
    x1 = rng.standard_normal((b, 3, n)).astype(np.float32)
    x2 = rng.standard_normal((b, 3, n)).astype(np.float32)
    i1 = rng.integers(0, n, size=(b, k, n)).astype(np.int32)
    i2 = rng.integers(0, n, size=(b, k, n)).astype(np.int32)
    i1[:, 0, :] = 0
    i2[:, 0, :] = 0
    gd1 = rng.standard_normal((b, k, n)).astype(np.float32)
    gd2 = rng.standard_normal((b, k, n)).astype(np.float32)
    args = [T(a, dev) for a in (x1, x2, gd1, gd2, i1, i2)]
    g1, g2 = ops.knn_backward_cuda(*args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r1, r2 = ops.knn_backward_cuda(*args)
    e1.record()
    torch.cuda.synchronize()
    print("hub neighbour: knn backward %.3f ms" % e0.elapsed_time(e1))
    assert torch.equal(g1, r1) and torch.equal(g2, r2)
    e1_, e2_ = oracle.knn_backward(x1, x2, gd1, gd2, i1, i2)
    b1, b2 = knn_backward_bound(x1, x2, gd1, gd2, i1, i2)
    assert_within_sum_order(N(g1), e1_, b1)
    assert_within_sum_order(N(g2), e2_, b2)


def test_knn_backward_gather_repeatable_and_entry_points(dev):
    """The atomics-free KNN backward (pcr_knn_backward_ws: pairs counting-
    sorted by neighbour, one gather per point) is bit-identical run to run,
    and both it and the atomic entry point (pcr_knn_backward) stay within the
    sum-order bound at the c2 shape, with unequal clouds (n != m) and the
    reference's 2 gd >= 20000 skip."""
    from pcr_amd import _lib, ops
    from pcr_amd.ops import _ptr, _stream
    b, n, m, k = 4, 1024, 900, 32
    x1, _, _ = gaussian_clouds(b, n, seed=24)
    x2, _, _ = gaussian_clouds(b, m, seed=25)
    _, _, i1, i2 = oracle.knn_forward(x1, x2, k)
    rng = np.random.default_rng(26)
    gd1 = rng.standard_normal((b, k, n)).astype(np.float32)
    gd2 = rng.standard_normal((b, k, m)).astype(np.float32)
    gd1[:, 7, ::3] = 10000.0
    args = [T(a, dev) for a in (x1, x2, gd1, gd2, i1, i2)]
    runs = [ops.knn_backward_cuda(*args) for _ in range(3)]
    for g in runs[1:]:
        assert torch.equal(g[0], runs[0][0]) and torch.equal(g[1], runs[0][1])
    e1, e2 = oracle.knn_backward(x1, x2, gd1, gd2, i1, i2)
    b1, b2 = knn_backward_bound(x1, x2, gd1, gd2, i1, i2)
    assert_within_sum_order(N(runs[0][0]), e1, b1)
    assert_within_sum_order(N(runs[0][1]), e2, b2)
    g1 = torch.full((b, 3, n), float("nan"), device=dev)
    g2 = torch.full((b, 3, m), float("nan"), device=dev)
    _lib.check(_lib.load().pcr_knn_backward(*[_ptr(a) for a in args], b, 3, n, m, k, _ptr(g1),
                                            _ptr(g2), _stream()), "knn_backward")
    assert_within_sum_order(N(g1), e1, b1)
    assert_within_sum_order(N(g2), e2, b2)


# ------------------------------------------------ ball query / grouping / PPF
def test_ball_query_grouping(dev):
    from pcr_amd import ops
    g = GOLDEN
    pts = T(g["bq_pts"], dev)
    idx = ops.ball_query(pts, pts, 0.3, 32)
    assert np.array_equal(N(idx), g["bq_idx"])
    grp = ops.grouping_forward(pts, idx)
    assert np.array_equal(N(grp), g["bq_grouped"])
    gx = ops.grouping_backward(T(g["grp_grad_y"], dev), idx, pts.shape[2])
    bound = grouping_backward_bound(g["grp_grad_y"], g["bq_idx"], pts.shape[2])
    assert_within_sum_order(N(gx), g["grp_grad_x"], bound)


def test_grouping_backward_model_shape(dev):
    """grouping_backward at the sph-dg model's ball query (u = 128, radius
    0.3) on 2048-point clouds (c3) against the oracle under the sum-order
    bound: the hot points receive up to hundreds of terms."""
    from pcr_amd import ops
    b, n, u, c = 2, 2048, 128, 6
    xyz, _, _ = gaussian_clouds(b, n, seed=31)
    xyz = (xyz / np.abs(xyz).max()).astype(np.float32)
    idx = oracle.ball_query(xyz, xyz, 0.3, u)
    gy = np.random.default_rng(32).standard_normal((b, c, n, u)).astype(np.float32)
    gx = ops.grouping_backward(T(gy, dev), T(idx, dev), n)
    exp = oracle.grouping_backward(gy, idx, n)
    assert_within_sum_order(N(gx), exp, grouping_backward_bound(gy, idx, n))


def test_ball_query_large(dev):
    from pcr_amd import ops
    xyz, _, _ = gaussian_clouds(2, 3000, seed=4)
    xyz = xyz * np.float32(0.4)
    idx = ops.ball_query(T(xyz, dev), T(xyz, dev), 0.3, 128)
    assert np.array_equal(N(idx), oracle.ball_query(xyz, xyz, 0.3, 128))


def test_local_ppf(dev):
    from pcr_amd import ops
    g = GOLDEN
    pts, nrm = T(g["bq_pts"], dev), T(g["bq_nrm"], dev)
    lp = ops.local_ppf_forward(pts, nrm, pts, nrm, T(g["bq_idx"], dev), kmajor=False)
    assert np.array_equal(N(lp), g["lppf_ball"], equal_nan=True)
    lk = ops.local_ppf_forward(pts, nrm, pts, nrm, T(g["lppf_knn_idx"], dev), kmajor=True)
    assert np.array_equal(N(lk), g["lppf_knn"], equal_nan=True)


def test_knn_local_ppf_fused(dev):
    from pcr_amd import ops
    xyz, nrm, _ = gaussian_clouds(3, 1024, seed=12)
    idx, ppf, dist = ops.knn_local_ppf(T(xyz, dev), T(nrm, dev), 32, want_dist=True)
    ed, ei = oracle.knn_dir(xyz, xyz, 32)
    assert np.array_equal(N(idx), ei)
    assert np.array_equal(N(dist), ed)
    ep = oracle.local_ppf(xyz, nrm, xyz, nrm, ei, kmajor=True, relative=True)
    assert np.array_equal(N(ppf), ep, equal_nan=True)


def test_global_ppf(dev):
    from pcr_amd import ops
    g = GOLDEN
    out = ops.spherical_ppf_forward(T(g["gppf_pts"], dev), T(g["gppf_cen"], dev),
                                    T(g["gppf_nrm"], dev), T(g["gppf_cnrm"], dev))
    assert np.array_equal(N(out), g["gppf_out"])
    assert (N(out)[:, :, 3] == 0).all()  # zero normal -> all-zero row


def test_center_gather(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(0)
    feat = rng.standard_normal((2, 6, 100)).astype(np.float32)
    grid = rng.standard_normal((2, 6, 512)).astype(np.float32)
    ind = rng.integers(-1, 512, (2, 100)).astype(np.int32)
    rel = N(ops.dgcnn_center_gather(T(feat, dev), T(grid, dev), T(ind, dev)))
    exp = feat - np.take_along_axis(grid, np.broadcast_to(np.maximum(ind, 0)[:, None, :],
                                                          feat.shape), axis=2)
    exp[np.broadcast_to((ind == -1)[:, None, :], feat.shape)] = 0
    assert np.array_equal(rel, exp)


def test_errors_are_raised(dev):
    from pcr_amd import ops
    x = torch.zeros((1, 3, 10), device=dev)
    with pytest.raises(RuntimeError, match="must be a float tensor"):
        ops.spherical_avg_voxelize_forward(x.double(), x, 8)
    with pytest.raises(RuntimeError, match="contiguous"):
        ops.knn_forward_cuda(x.transpose(1, 2), x, 4)
    with pytest.raises(RuntimeError, match="too large"):
        ops.spherical_avg_voxelize_forward(x, x, 300)


def test_sph_devox_backward_irregular_corners(dev):
    """The wave-sorted segmented path takes corner sets of the spherical
    pattern; anything else (arbitrary corners, -1 points, corners past the
    hot window) falls back to per-point atomics.  Both against the oracle."""
    from pcr_amd import ops
    rng = np.random.default_rng(7)
    b, c, n, r = 2, 5, 3000, 16
    xyz, _, feat = gaussian_clouds(b, n, seed=8, c=c)
    nc = oracle.normalize_sph(xyz)
    grid, gind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    _, inds, wgts = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, gind)
    inds = inds.copy()
    wgts = wgts.copy()
    pick = rng.choice(n, 400, replace=False)
    inds[0][:, pick[:200]] = rng.integers(0, r ** 3, size=(8, 200))       # arbitrary corners
    inds[1][:, pick[200:300]] = rng.integers(0, r * r + 8 * r, size=(8, 100))
    inds[1][0, pick[300:]] = -1                                         # skipped points
    gy = rng.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.spherical_trilinear_devoxelize_backward(T(gy, dev), T(inds, dev), T(wgts, dev), r)
    exp = oracle.devoxelize_backward(gy, inds, wgts, r, spherical=True)
    assert_within_sum_order(N(gx), exp,
                            devox_backward_bound(gy, inds, wgts, r ** 3, skip_neg=True))


@pytest.mark.parametrize("b,m,n,radius,u,scale", [
    (3, 1024, 1024, 0.3, 128, 0.35),   # the sph-dg model's BallQuery(0.3, 128) at c2
    (2, 700, 1500, 0.3, 16, 0.35),     # centres != points, u reached early (index-order cut)
    (2, 513, 2048, 0.2, 128, 0.35),    # c3 per-cloud size, ragged centre count
    (1, 64, 77, 0.9, 200, 0.35),       # u > n: padding with the first hit
    (1, 100, 300, 0.05, 8, 1.0),       # sparse: many centres with no hit (all-0 rows)
    (2, 300, 4000, 0.3, 128, 0.35),    # near the hit-bit kernel's LDS limit (~4.9k points)
    (2, 256, 9000, 0.3, 64, 0.35),     # beyond the hit-bit kernel's LDS budget: the scan kernel
])
def test_ball_query_paths(dev, b, m, n, radius, u, scale):
    """pcr_ball_query's hit-bit kernel (and the per-centre scan past its LDS
    budget) against ball_query.cu:30-49 as the oracle restates it."""
    from pcr_amd import ops
    rng = np.random.default_rng(m + n + u)
    pts = (rng.standard_normal((b, 3, n)) * scale).astype(np.float32)
    ctr = (rng.standard_normal((b, 3, m)) * scale).astype(np.float32)
    ctr[:, :, :min(m, n) // 4] = pts[:, :, :min(m, n) // 4]   # centres on points: d2 = 0 excluded
    pts[:, :, 5:9] = pts[:, :, 1:2]                             # duplicates
    idx = ops.ball_query(T(ctr, dev), T(pts, dev), radius, u)
    assert np.array_equal(N(idx), oracle.ball_query(ctr, pts, radius, u))


@pytest.mark.parametrize("b,n,c,r", [(2, 1500, 67, 2), (2, 700, 5, 3), (1, 3000, 130, 4),
                                     (2, 1025, 64, 7), (1, 4097, 16, 16), (1, 2048, 64, 64)])
def test_sph_devox_forward_corner_staging(dev, b, n, c, r):
    """The LDS-staged spherical devox forward (devox_fwd_sph_lds_kernel):
    tiny grids whose 80 corner slots alias or run past r^3, channel counts
    across the 64-channel groups, ragged point counts, dropped points
    (g_inds = -1) and invalid voxel indices (>= r^3: corners outside the
    staged set, read from global memory and bounds-checked) -- bit-exact
    against the oracle."""
    from pcr_amd import ops
    xyz, _, _ = gaussian_clouds(b, n, seed=40 + r)
    nc = oracle.normalize_sph(xyz)
    ind = np.stack([oracle.sph_index(nc[i], r) for i in range(b)]).astype(np.int32)
    ind[:, 3::97] = -1
    if r >= 4:
        ind[0, 5::113] = r ** 3 + 7 * r  # invalid: corners beyond the 80-slot set
    grid = np.random.default_rng(41).standard_normal((b, c, r ** 3)).astype(np.float32)
    outs, inds, wgts = ops.spherical_trilinear_devoxelize_forward(r, True, T(nc, dev),
                                                                  T(grid, dev), T(ind, dev))
    eo, ei, ew = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    # out-of-range corners contribute 0 in both (the reference would read
    # out of bounds there)
    assert np.array_equal(N(outs), eo)
