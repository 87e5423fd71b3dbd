"""Clouds beyond the 4096-point single-workgroup paths (BASELINE c5: 8 x
65,536 points, k = 64, r = 64): normalisation, spherical / cube
voxelisation on the global-atomic path, devoxelisation and KNN, against the
oracle at sizes it finishes in seconds, plus size-independent properties at
the full c5 cloud size.  The large-cloud voxelisers sort the points by voxel
(a hand-written counting sort; voxels of more than 64 points by a stable
workgroup radix sort) and sum each voxel in ascending point order, the
oracle's order, so their grids are bit-exact."""
import numpy as np
import pytest

import oracle
from clouds import gaussian_clouds

pytestmark = pytest.mark.gpu

# voxel means summed in atomic (arbitrary) order, as the reference does
SUM_ORDER_TOL = 1e-5


def T(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def test_normalize_large(dev):
    from pcr_amd import ops
    xyz, _, _ = gaussian_clouds(2, 20000, seed=41)
    xyz = xyz * np.float32(2.5) + np.float32(0.7)
    got = ops.spherical_normalize(T(xyz, dev))
    assert np.array_equal(N(got), oracle.normalize_sph(xyz))


def test_sph_vox_large(dev):
    from pcr_amd import ops
    xyz, _, feat = gaussian_clouds(2, 20000, seed=42, c=8)
    nc = oracle.normalize_sph(xyz)
    out, ind, cnt = ops.spherical_avg_voxelize_forward(T(feat, dev), T(nc, dev), 64)
    eo, ei, ec = oracle.spherical_avg_voxelize_forward(feat, nc, 64)
    assert np.array_equal(N(ind), ei)
    assert np.array_equal(N(cnt), ec.reshape(N(cnt).shape))
    assert np.array_equal(N(out).reshape(eo.shape), eo)


@pytest.mark.parametrize("kind", ["one_voxel_20pct", "many_heavy_voxels"])
def test_sph_vox_large_heavy_voxels(dev, kind):
    """A 65,536-point cloud (BASELINE c5 size, r = 64) whose points pile into
    few voxels: 20% of them duplicated at one location, or 100 locations
    with 300 copies each.  Segments past 64 points are sorted by the stable
    workgroup radix sort (vox_seg_sort_kernel) instead of the O(m^2) rank
    scan; ind / cnt / grid bit-exact vs the oracle, time printed."""
    import torch
    from pcr_amd import ops
    b, n, c, r = 2, 65536, 8, 64
    xyz, _, feat = gaussian_clouds(b, n, seed=44, c=c)
    if kind == "one_voxel_20pct":
        xyz[:, :, 1000:1000 + n // 5] = xyz[:, :, 7:8]
    else:
        for h in range(100):
            xyz[:, :, 2000 + h * 300:2000 + (h + 1) * 300] = xyz[:, :, h:h + 1]
    nc = oracle.normalize_sph(xyz)
    tf, tn = T(feat, dev), T(nc, dev)
    out, ind, cnt = ops.spherical_avg_voxelize_forward(tf, tn, r)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.spherical_avg_voxelize_forward(tf, tn, r)
    e1.record()
    torch.cuda.synchronize()
    print("%s: sph voxelize %.3f ms, largest voxel %d points" %
          (kind, e0.elapsed_time(e1), int(N(cnt).max())))
    eo, ei, ec = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    assert np.array_equal(N(ind), ei)
    assert np.array_equal(N(cnt), ec.reshape(N(cnt).shape))
    assert np.array_equal(N(out).reshape(eo.shape), eo)


def test_cube_vox_large(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(43)
    b, n, c, r = 2, 12000, 5, 32
    coords = rng.integers(0, r, size=(b, 3, n)).astype(np.int32)
    coords[:, :, :7] = -1  # out-of-range voxel coordinates
    feat = rng.standard_normal((b, c, n)).astype(np.float32)
    out, ind, cnt = ops.avg_voxelize_forward(T(feat, dev), T(coords, dev), r)
    eo, ei, ec = oracle.avg_voxelize_forward(feat, coords, r)
    assert np.array_equal(N(ind), ei)
    assert np.array_equal(N(cnt), ec.reshape(N(cnt).shape))
    assert np.array_equal(N(out).reshape(eo.shape), eo)


def test_sph_devox_large(dev):
    from pcr_amd import ops
    xyz, _, feat = gaussian_clouds(2, 20000, seed=44, c=4)
    nc = oracle.normalize_sph(xyz)
    grid, gind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, 64)
    outs, inds, wgts = ops.spherical_trilinear_devoxelize_forward(
        64, False, T(nc, dev), T(grid.reshape(2, 4, -1), dev), T(gind, dev))
    eo, ei, ew = oracle.spherical_trilinear_devoxelize_forward(64, nc, grid, gind)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    assert np.abs(N(outs) - eo).max() <= SUM_ORDER_TOL


def test_knn_large_k64(dev):
    from pcr_amd import ops
    xyz, nrm, _ = gaussian_clouds(1, 8192, seed=45)
    d1, d2, i1, i2 = ops.knn_forward_cuda(T(xyz, dev), T(xyz, dev), 64)
    e = oracle.knn_forward(xyz, xyz, 64)
    for got, exp in zip((d1, d2, i1, i2), e):
        assert np.array_equal(N(got), exp)
    idx, ppf, _ = ops.knn_local_ppf(T(xyz, dev), T(nrm, dev), 64)
    assert np.array_equal(N(idx), e[2])
    ep = oracle.local_ppf(xyz, nrm, xyz, nrm, e[2], kmajor=True, relative=True)
    assert np.array_equal(N(ppf), ep, equal_nan=True)


@pytest.mark.parametrize("n,k", [(4097, 32), (6000, 16), (9000, 64)])
def test_knn_large_sorted_path(dev, n, k):
    """Clouds past the single-workgroup sort: global counting sort, then the
    selection (k <= 32) or block kernels, bit-exact."""
    from pcr_amd import ops
    xyz, nrm, _ = gaussian_clouds(2, n, seed=n + k)
    xyz[1, :, 50:90] = xyz[1, :, 50:51]          # duplicates
    xyz[0, :, 7] = np.nan                        # a NaN point
    idx, ppf, dist = ops.knn_local_ppf(T(xyz, dev), T(nrm, dev), k, want_dist=True)
    ed, ei = oracle.knn_dir(xyz, xyz, k)
    assert np.array_equal(N(idx), ei)
    assert np.array_equal(N(dist), ed)


def test_knn_large_two_sets(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(12)
    x1 = rng.standard_normal((1, 3, 7000)).astype(np.float32)
    x2 = (rng.standard_normal((1, 3, 5000)) * 0.5 + 0.3).astype(np.float32)
    got = ops.knn_forward_cuda(T(x1, dev), T(x2, dev), 32)
    for a, b in zip(got, oracle.knn_forward(x1, x2, 32)):
        assert np.array_equal(N(a), b)


def test_c5_cloud_properties(dev):
    """One c5-sized cloud (65,536 points, k = 64, r = 64, C = 64):
    size-independent properties of the whole path."""
    import torch
    from pcr_amd import ops
    n, k, r, c = 65536, 64, 64, 64
    xyz, nrm, feat = gaussian_clouds(1, n, seed=46, c=c)
    tx, tn, tf = T(xyz, dev), T(nrm, dev), T(feat, dev)
    idx, ppf, dist = ops.knn_local_ppf(tx, tn, k, want_dist=True)
    i, d = N(idx), N(dist)
    assert ((i >= 0) & (i < n)).all()
    assert (np.diff(d, axis=1) >= 0).all()                      # ascending per point
    assert (d[:, 0] == 0).all()                                 # self (or a duplicate)
    samp = np.random.default_rng(0).choice(n, 64, replace=False)
    ref_d, ref_i = oracle.knn_dir(np.ascontiguousarray(xyz[:, :, samp]), xyz, k)
    assert np.array_equal(d[0][:, samp], ref_d[0])             # spot-check exact lists
    assert np.array_equal(i[0][:, samp], ref_i[0])
    nc = ops.spherical_normalize(tx)
    out, ind, cnt = ops.spherical_avg_voxelize_forward(tf, nc, r)
    ind_, cnt_ = N(ind), N(cnt).reshape(1, -1)
    valid = ind_ >= 0
    assert cnt_.sum() == valid.sum()
    assert np.array_equal(np.bincount(ind_[valid], minlength=r ** 3), cnt_[0])
    grid = N(out).reshape(1, c, -1)
    assert (grid[:, :, cnt_[0] == 0] == 0).all()
    torch.cuda.synchronize()


def test_sph_vox_large_without_feature_copy(dev):
    """Workspace sized by pcr_voxelize_workspace_size (no channel count):
    the direct-gather variant, same bits as the point-major one."""
    import torch
    from pcr_amd import _lib, ops
    from pcr_amd.ops import _ptr
    xyz, _, feat = gaussian_clouds(2, 9000, seed=47, c=6)
    nc = oracle.normalize_sph(xyz)
    b, c, n, r = 2, 6, 9000, 32
    lib = _lib.load()
    small = lib.pcr_voxelize_workspace_size(b, n, r)
    assert lib.pcr_voxelize_workspace_size_c(b, c, n, r) > small
    ws = torch.empty(small, dtype=torch.uint8, device=dev)
    tf, tc = T(feat, dev), T(nc, dev)
    out = torch.empty((b, c, r ** 3), device=dev)
    ind = torch.empty((b, n), dtype=torch.int32, device=dev)
    cnt = torch.empty((b, r ** 3), dtype=torch.int32, device=dev)
    _lib.check(lib.pcr_spherical_avg_voxelize_forward(
        _ptr(tf), _ptr(tc), b, c, n, r, _ptr(out), _ptr(ind), _ptr(cnt), _ptr(ws), ws.numel(),
        torch.cuda.current_stream().cuda_stream), "vox")
    ref = ops.spherical_avg_voxelize_forward(tf, tc, r)
    eo, _, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    assert np.array_equal(N(out).reshape(eo.shape), eo)
    assert torch.equal(out, ref[0]) and torch.equal(ind, ref[1]) and torch.equal(cnt, ref[2])


@pytest.mark.parametrize("shape", ["gauss", "clusters"])
def test_knn_c5_k64_query_sample_vs_oracle(dev, shape):
    """BASELINE c5 KNN (65,536 points, k = 64): 1,024 sampled queries per
    cloud bit-exact (indices and distances) against the oracle's reference
    scan, for Gaussian clouds and for tight clusters with a sparse halo
    (queries whose k-th distance is far below D_q, and outliers whose
    neighbours are far away) -- the large-cloud selection's two count rounds."""
    from pcr_amd import ops
    n, k = 65536, 64
    xyz, nrm, _ = gaussian_clouds(2, n, seed=47)
    if shape == "clusters":
        rng = np.random.default_rng(48)
        cen = rng.standard_normal((2, 3, 8)).astype(np.float32) * 3
        lab = rng.integers(0, 8, (2, n))
        for b in range(2):
            xyz[b] = cen[b][:, lab[b]] + 0.02 * xyz[b]
        xyz[:, :, :200] *= 40  # sparse halo / outliers
    idx, _, dist = ops.knn_local_ppf(T(xyz, dev), T(nrm, dev), k, want_dist=True)
    i, d = N(idx), N(dist)
    samp = np.random.default_rng(49).choice(n, 1024, replace=False)
    samp[:64] = np.arange(64)  # include halo points
    ref_d, ref_i = oracle.knn_dir(np.ascontiguousarray(xyz[:, :, samp]), xyz, k)
    assert np.array_equal(i[:, :, samp], ref_i)
    assert np.array_equal(d[:, :, samp], ref_d)
