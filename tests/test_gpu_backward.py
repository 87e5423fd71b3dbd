"""GPU parity of the backward passes at the resolutions and shapes the models
run (BASELINE c3: 2048 points, r = 32, C = 64), one test per kernel branch.

Cube trilinear devoxelize backward (trilinear_devox.cu:120-163) has three
launch shapes in pcr_devoxelize_backward (csrc/devoxelize.hip):
  * r^3 <= 2048 (r = 8):  the grid window covers r^3, several channels per
    workgroup (golden fixture, tests/test_gpu_ops.py);
  * 2048 < r^3 <= 32768 (r = 16, 32): one channel's whole grid in LDS, one
    channel per workgroup ("lds_whole_grid");
  * r^3 > 32768 (r = 64): a 20k-voxel LDS window plus global atomics for the
    corners past it ("window_atomics").
With the pcr_devoxelize_backward_workspace_size_r workspace (what ops.py
passes), r <= 32 instead takes the atomics-free gather: the (point, corner)
pairs counting-sorted by voxel once per cloud, one thread per voxel
summing its segment ("voxel_gather"; test_cube_devox_backward_entry_points
covers both it and the LDS kernel at r = 16 / 32).
Scatter results are compared against the oracle with the fp32 sum-order
bound of tests/sumorder.py; the gather backward (avg voxelize) is bit-exact.
"""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds
from sumorder import assert_within_sum_order, devox_backward_bound

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def cube_coords(b, n, r, seed):
    """Continuous voxel coords in [0, r-1] as Voxelization produces them
    (voxelization.py:18-31), with exact lattice points, the r-1 face and the
    0 face among them."""
    rng = np.random.default_rng(seed)
    cc = rng.uniform(0, r - 1, (b, 3, n)).astype(np.float32)
    cc[:, :, :16] = rng.integers(0, r, (b, 3, 16)).astype(np.float32)
    cc[:, 0, 16:24] = r - 1
    cc[:, 1, 24:32] = 0.0
    return np.ascontiguousarray(cc)


@pytest.mark.parametrize("r,branch", [(16, "voxel_gather"), (32, "voxel_gather"),
                                      (64, "window_atomics")])
def test_cube_devox_backward_branches(dev, r, branch):
    from pcr_amd import ops
    b, n = 2, 2048
    c = 67 if r < 64 else 21  # not a multiple of any channel group
    cc = cube_coords(b, n, r, seed=r)
    rng = np.random.default_rng(100 + r)
    grid = rng.standard_normal((b, c, r ** 3)).astype(np.float32)
    outs, inds, wgts = ops.trilinear_devoxelize_forward(r, True, T(cc, dev), T(grid, dev))
    eo, ei, ew = oracle.trilinear_devoxelize_forward(r, cc, grid)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    assert np.abs(N(outs) - eo).max() <= 1e-5
    gy = rng.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.trilinear_devoxelize_backward(T(gy, dev), inds, wgts, r)
    exp = oracle.devoxelize_backward(gy, ei, ew, r, spherical=False)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3))


def test_cube_devox_backward_clustered(dev):
    """r = 32 with every point inside a few voxels: long per-voxel sums (the
    LDS float-atomic contention case) still within the sum-order bound."""
    from pcr_amd import ops
    b, n, c, r = 2, 2048, 64, 32
    rng = np.random.default_rng(5)
    cc = (rng.integers(10, 13, (b, 3, n)) + rng.uniform(0, 1, (b, 3, n)) * 0.999).astype(
        np.float32)
    _, ei, ew = oracle.trilinear_devoxelize_forward(r, cc, np.zeros((b, c, r ** 3), np.float32))
    gy = rng.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.trilinear_devoxelize_backward(T(gy, dev), T(ei, dev), T(ew, dev), r)
    exp = oracle.devoxelize_backward(gy, ei, ew, r, spherical=False)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3))


def _sph_setup(b, n, c, r, seed):
    xyz, _, feat = gaussian_clouds(b, n, seed=seed, c=c)
    nc = oracle.normalize_sph(xyz)
    grid, gind, cnt = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    return nc, feat, grid, gind, cnt


def test_sph_devox_backward_c3_shape(dev):
    """Spherical devox backward at the c3 per-cloud shape (N = 2048, r = 32,
    C = 64, B = 4): the wave-sorted segmented path."""
    from pcr_amd import ops
    b, n, c, r = 4, 2048, 64, 32
    nc, _, grid, gind, _ = _sph_setup(b, n, c, r, seed=31)
    outs, inds, wgts = ops.spherical_trilinear_devoxelize_forward(r, True, T(nc, dev),
                                                                  T(grid, dev), T(gind, dev))
    eo, ei, ew = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, gind)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    assert np.array_equal(N(outs), eo)
    gy = np.random.default_rng(32).standard_normal((b, c, n)).astype(np.float32)
    gx = ops.spherical_trilinear_devoxelize_backward(T(gy, dev), inds, wgts, r)
    exp = oracle.devoxelize_backward(gy, ei, ew, r, spherical=True)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3, skip_neg=True))


@pytest.mark.parametrize("b,n,c,r", [(2, 1024, 64, 32), (2, 2048, 16, 16), (1, 4096, 8, 64)])
def test_sph_devox_backward_sum_order(dev, b, n, c, r):
    """The shapes of the older 1e-3 test, now at the sum-order bound."""
    from pcr_amd import ops
    nc, _, grid, gind, _ = _sph_setup(b, n, c, r, seed=5)
    _, ei, ew = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, gind)
    gy = np.random.default_rng(3).standard_normal((b, c, n)).astype(np.float32)
    gx = ops.spherical_trilinear_devoxelize_backward(T(gy, dev), T(ei, dev), T(ew, dev), r)
    exp = oracle.devoxelize_backward(gy, ei, ew, r, spherical=True)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3, skip_neg=True))


@pytest.mark.parametrize("with_ws", [False, True])
def test_sph_devox_backward_entry_points(dev, with_ws):
    """Both C entry points at the c3 per-cloud shape: pcr_devoxelize_backward
    (each workgroup sorts every 64 points by corner set) and
    pcr_devoxelize_backward_ws (each cloud's points sorted once, the corner
    data read in that order), against the oracle at the sum-order bound."""
    from pcr_amd import _lib
    from pcr_amd.ops import _ptr, _stream
    b, n, c, r = 3, 2048, 24, 32
    nc, _, grid, gind, _ = _sph_setup(b, n, c, r, seed=41)
    _, ei, ew = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, gind)
    gy = np.random.default_rng(42).standard_normal((b, c, n)).astype(np.float32)
    tg, ti, tw = T(gy, dev), T(ei, dev), T(ew, dev)
    gx = torch.full((b, c, r ** 3), float("nan"), device=dev)
    lib = _lib.load()
    if with_ws:
        ws = torch.empty(lib.pcr_devoxelize_backward_workspace_size(b, n), dtype=torch.uint8,
                         device=dev)
        rc = lib.pcr_devoxelize_backward_ws(_ptr(tg), _ptr(ti), _ptr(tw), b, c, n, r, 1,
                                            _ptr(gx), _ptr(ws), ws.numel(), _stream())
    else:
        rc = lib.pcr_devoxelize_backward(_ptr(tg), _ptr(ti), _ptr(tw), b, c, n, r, 1, _ptr(gx),
                                         _stream())
    _lib.check(rc, "devoxelize_backward")
    exp = oracle.devoxelize_backward(gy, ei, ew, r, spherical=True)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3, skip_neg=True))


def test_sph_avg_vox_backward_c3_shape(dev):
    """spherical_avg_voxelize backward (spherical_vox.cu:139-163) at the c3
    per-cloud shape: a gather, bit-exact (dropped points get 0)."""
    from pcr_amd import ops
    b, n, c, r = 4, 2048, 64, 32
    nc, feat, _, gind, cnt = _sph_setup(b, n, c, r, seed=33)
    gy = np.random.default_rng(34).standard_normal((b, c, r ** 3)).astype(np.float32)
    gx = ops.spherical_avg_voxelize_backward(T(gy, dev), T(gind, dev), T(cnt, dev))
    assert np.array_equal(N(gx), oracle.avg_voxelize_backward(gy, gind, cnt))
    assert (N(gx)[np.broadcast_to((gind == -1)[:, None, :], gx.shape)] == 0).all()


@pytest.mark.parametrize("v0", [-1.5, float("nan"), float("-inf")])
def test_sph_avg_vox_backward_dropped_points_positive_zero(dev, v0):
    """Points the voxelisation drops (ind = -1) keep the +0 the reference's
    zero-initialised grad_x holds (spherical_vox.cu:153-156), whatever
    grad_y[voxel 0] is: the sorted gather must not write grad_y[0] * 0 there
    (-0 for a negative value, NaN for inf / NaN)."""
    from pcr_amd import ops
    b, n, c, r = 2, 2048, 20, 32
    nc, _, _, gind, cnt = _sph_setup(b, n, c, r, seed=36)
    gind = gind.copy()
    gind[:, ::7] = -1  # about 1 in 7 points dropped
    gy = np.random.default_rng(37).standard_normal((b, c, r ** 3)).astype(np.float32)
    gy[:, :, 0] = v0
    gx = N(ops.spherical_avg_voxelize_backward(T(gy, dev), T(gind, dev), T(cnt, dev)))
    exp = oracle.avg_voxelize_backward(gy, gind, cnt)
    drop = np.broadcast_to((gind == -1)[:, None, :], gx.shape)
    assert (gx[drop] == 0).all() and not np.signbit(gx[drop]).any()
    assert np.array_equal(gx[~drop], exp[~drop], equal_nan=True)


def test_cube_avg_vox_backward_c3_shape(dev):
    from pcr_amd import ops
    b, n, c, r = 4, 2048, 64, 32
    rng = np.random.default_rng(35)
    vc = rng.integers(0, r, (b, 3, n)).astype(np.int32)
    feat = rng.uniform(-1, 1, (b, c, n)).astype(np.float32)
    out, ind, cnt = ops.avg_voxelize_forward(T(feat, dev), T(vc, dev), r)
    eo, ei, ec = oracle.avg_voxelize_forward(feat, vc, r)
    assert np.array_equal(N(ind), ei)
    assert np.array_equal(N(cnt), ec)
    assert np.array_equal(N(out), eo)
    gy = rng.standard_normal((b, c, r ** 3)).astype(np.float32)
    gx = ops.avg_voxelize_backward(T(gy, dev), ind, cnt)
    assert np.array_equal(N(gx), oracle.avg_voxelize_backward(gy, ei, ec))


def test_cube_vox_forward_repeated(dev):
    """The prep kernel zeroes its occupancy bitmap and then sets bits with LDS
    atomics; on the cube path nothing else separated the two, so a slow
    wave's zeroing could erase a fast wave's bit (a voxel then lost its bit
    and its points joined the next segment: ~13% of runs at this shape).
    Repeated runs must all match the oracle."""
    from pcr_amd import ops
    b, n, c, r = 4, 2048, 16, 32
    rng = np.random.default_rng(36)
    vc = rng.integers(0, r, (b, 3, n)).astype(np.int32)
    feat = rng.uniform(-1, 1, (b, c, n)).astype(np.float32)
    eo, ei, ec = oracle.avg_voxelize_forward(feat, vc, r)
    tf, tv = T(feat, dev), T(vc, dev)
    ecnt = torch.from_numpy(ec).to(dev)
    bad = 0
    for _ in range(60):
        out, ind, cnt = ops.avg_voxelize_forward(tf, tv, r)
        bad += int(not torch.equal(cnt, ecnt))
    assert bad == 0, "%d of 60 runs gave wrong voxel counts" % bad
    assert np.array_equal(N(out), eo) and np.array_equal(N(ind), ei)


@pytest.mark.parametrize("r", [8, 32, 33, 40])
def test_cube_devox_forward_row_kernel(dev, r):
    """Cube devox forward: r <= 32 stages each channel row in LDS
    (devox_fwd_cube_row_kernel), larger grids gather from global memory; both
    bit-exact against the oracle (same corners, same wsum8 order)."""
    from pcr_amd import ops
    b, n, c = 2, 2048, 12
    rng = np.random.default_rng(50 + r)
    cc = rng.uniform(0, r - 1, (b, 3, n)).astype(np.float32)
    cc[:, :, :8] = np.floor(cc[:, :, :8])  # points exactly on cell corners
    grid = rng.standard_normal((b, c, r, r, r)).astype(np.float32)
    outs, inds, wgts = ops.trilinear_devoxelize_forward(r, True, T(cc, dev), T(grid, dev))
    eo, ei, ew = oracle.trilinear_devoxelize_forward(r, cc, grid)
    assert np.array_equal(N(inds), ei)
    assert np.array_equal(N(wgts), ew)
    assert np.array_equal(N(outs), eo)


@pytest.mark.parametrize("r,n", [(5, 1500), (16, 1500), (32, 1500), (16, 3000), (24, 600)])
@pytest.mark.parametrize("path", ["lds_atomics", "voxel_gather", "small_ws"])
def test_cube_devox_backward_entry_points(dev, r, n, path):
    """Cube grads through the C entry points: pcr_devoxelize_backward (LDS
    float atomics), pcr_devoxelize_backward_ws with the _size_r workspace
    (voxel-sorted gather) and with only the (b, n) workspace (falls back to
    the LDS kernel).  Includes corners outside [0, r^3) (dropped by every
    path) and a cloud with all points in one cell (one long segment).
    The gather stages the gradient rows in LDS up to ~2.7k points
    (devox_cube_gather_lds_kernel, n = 1500) and reads them from global
    memory beyond (devox_cube_gather_kernel, n = 3000)."""
    from pcr_amd import _lib
    from pcr_amd.ops import _ptr, _stream
    b, c = 3, 19
    cc = cube_coords(b, n, r, seed=60 + r)
    cc[2] = (r // 2 + 0.25 + 0.5 * np.random.default_rng(61).uniform(0, 1, (3, n))).astype(
        np.float32)
    _, ei, ew = oracle.trilinear_devoxelize_forward(r, cc, np.zeros((b, c, r ** 3), np.float32))
    ei = ei.copy()
    ei[0, 3, :7] = r ** 3 + 5
    ei[1, 6, 10:13] = -4
    gy = np.random.default_rng(62 + r).standard_normal((b, c, n)).astype(np.float32)
    tg, ti, tw = T(gy, dev), T(ei, dev), T(ew, dev)
    gx = torch.full((b, c, r ** 3), float("nan"), device=dev)
    lib = _lib.load()
    if path == "lds_atomics":
        rc = lib.pcr_devoxelize_backward(_ptr(tg), _ptr(ti), _ptr(tw), b, c, n, r, 0, _ptr(gx),
                                         _stream())
    else:
        size_r = lib.pcr_devoxelize_backward_workspace_size_r(b, n, r, 0)
        base = lib.pcr_devoxelize_backward_workspace_size(b, n)
        if path == "voxel_gather":
            size = size_r
        else:
            # just below what the gather needs, so the call must take the LDS
            # kernel (at r = 5 the gather needs less than the base size, so
            # no valid workspace can force the fallback there)
            if size_r - 256 < base:
                pytest.skip("r=%d n=%d: the gather fits in the base workspace" % (r, n))
            size = size_r - 256
        ws = torch.empty(size, dtype=torch.uint8, device=dev)
        rc = lib.pcr_devoxelize_backward_ws(_ptr(tg), _ptr(ti), _ptr(tw), b, c, n, r, 0,
                                            _ptr(gx), _ptr(ws), ws.numel(), _stream())
    _lib.check(rc, "devoxelize_backward")
    keep = (ei >= 0) & (ei < r ** 3)
    exp = oracle.devoxelize_backward(gy, np.where(keep, ei, 0), np.where(keep, ew, 0), r,
                                     spherical=False)
    assert_within_sum_order(N(gx), exp, devox_backward_bound(gy, ei, ew, r ** 3))


def test_cube_devox_backward_bitwise_repeatable(dev):
    """The cube gather's pairs are placed by one wave in a fixed order
    (devox_cube_order_kernel), so the gradient grid is bit-identical from run
    to run at the c3 cube shape (one cloud's worth of waves per workgroup)."""
    from pcr_amd import ops
    b, n, c, r = 16, 2048, 64, 32
    cc = cube_coords(b, n, r, seed=70)
    _, ei, ew = oracle.trilinear_devoxelize_forward(r, cc, np.zeros((b, c, r ** 3), np.float32))
    gy = T(np.random.default_rng(71).standard_normal((b, c, n)).astype(np.float32), dev)
    ti, tw = T(ei, dev), T(ew, dev)
    ref = ops.trilinear_devoxelize_backward(gy, ti, tw, r).clone()
    for _ in range(10):
        assert torch.equal(ops.trilinear_devoxelize_backward(gy, ti, tw, r), ref)
