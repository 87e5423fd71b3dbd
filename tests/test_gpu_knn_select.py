"""Parity of the KNN selection kernel's special paths against the oracle
(bit-exact): the histogram / cut / collect / rank path, the exact LDS
insertion fallback (too many collected keys, no finite bound), ties,
unfilled slots, NaN and far-away points, ragged sizes, k = 1 .. 32."""
import numpy as np
import pytest

import oracle
from clouds import edge_clouds_for_knn, gaussian_clouds

pytestmark = pytest.mark.gpu


def T(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def check_sorted(dev, xyz, nrm, k, exp_idx):
    """The extractor's selection (pcr_knn_prepare + pcr_knn_select_ppf: ids
    in sorted query order, clouds of <= 1024 points through the transposed
    knn_wsel_kernel) on the same cloud, every output poisoned first."""
    import torch
    from pcr_amd import _lib
    from pcr_amd.ops import _ptr, _stream
    b, _, n = xyz.shape
    tx, tn = T(xyz, dev), T(nrm, dev)
    lib = _lib.load()
    ws = torch.full((lib.pcr_knn_workspace_size(b, n, n),), 0xA5, dtype=torch.uint8, device=dev)
    idx = torch.full((b, k, n), -7, dtype=torch.int32, device=dev)
    ppf = torch.full((b, 4, k, n), float("nan"), device=dev)
    _lib.check(lib.pcr_knn_prepare(_ptr(tx), b, n, _ptr(ws), ws.numel(), _stream()), "prepare")
    _lib.check(lib.pcr_knn_select_ppf(_ptr(tx), _ptr(tn), b, n, k, 1, _ptr(idx), _ptr(ppf),
                                      _ptr(ws), ws.numel(), _stream()), "select_ppf")
    torch.cuda.synchronize()
    got = N(idx)
    bad = np.argwhere(got != exp_idx)
    assert bad.size == 0, "sorted-path idx differs at %d places, first %s: got %s exp %s" % (
        len(bad), bad[:3].tolist(), got[tuple(bad[0])], exp_idx[tuple(bad[0])])


def check_self(dev, xyz, k):
    """knn_forward_cuda(xyz, xyz, k) and the fused knn_local_ppf vs the oracle."""
    from pcr_amd import ops
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    d1, d2, i1, i2 = ops.knn_forward_cuda(T(xyz, dev), T(xyz, dev), k)
    e = oracle.knn_forward(xyz, xyz, k)
    for name, got, exp in zip(("d1", "d2", "i1", "i2"), (d1, d2, i1, i2), e):
        assert np.array_equal(N(got), exp, equal_nan=True), name
    nrm = np.ascontiguousarray(np.roll(xyz, 1, axis=1))
    idx, ppf, dist = ops.knn_local_ppf(T(xyz, dev), T(nrm, dev), k, want_dist=True)
    assert np.array_equal(N(idx), e[2])
    assert np.array_equal(N(dist), e[0])
    ep = oracle.local_ppf(xyz, nrm, xyz, nrm, e[2], kmajor=True, relative=True)
    assert np.array_equal(N(ppf), ep, equal_nan=True)
    if k <= 32 and xyz.shape[2] <= 2048:
        check_sorted(dev, xyz, nrm, k, e[2])


@pytest.mark.parametrize("k", [1, 7, 16, 31, 32])
def test_select_k_values(dev, k):
    xyz, _, _ = gaussian_clouds(3, 1024, seed=20 + k)
    check_self(dev, xyz, k)


@pytest.mark.parametrize("n", [1000, 65, 129, 700, 1025, 2048, 3001, 4096])
def test_select_ragged_sizes(dev, n):
    """<= 1024 points: the LDS candidate cache with byte fields; <= 2048
    (BASELINE c3): the 2048-candidate cache with 16-bit fields; beyond: the
    global-memory sweep with per-block box tests."""
    xyz, _, _ = gaussian_clouds(2, n, seed=n)
    check_self(dev, xyz, 32)


def test_select_cached_2k_duplicates_and_k16(dev):
    xyz, _, _ = gaussian_clouds(2, 2048, seed=77)
    xyz[0, :, 500:700] = xyz[0, :, 500:501]  # fallback blocks past the LDS cache
    check_self(dev, xyz, 32)
    check_self(dev, xyz, 16)


@pytest.mark.parametrize("n", [1024, 2048, 3001])
def test_select_outlier_refined_cut(dev, n):
    """Far outliers facing a compact cloud: their distances to the bulk fall
    into one or two quarter-octave bins (far more than the 88-key capacity),
    so their query blocks recount inside the cut bin with 1/64-octave bins
    (the refinement pass) instead of taking the insertion fallback."""
    xyz, _, _ = gaussian_clouds(2, n, seed=n + 5)
    xyz[0, :, 7] = (30.0, 0.0, 0.0)
    xyz[0, :, n // 2] = (0.0, -12.0, 5.0)
    xyz[1, :, n - 1] = (8.0, 8.0, 8.0)
    check_self(dev, xyz, 32)
    check_self(dev, xyz, 16)


def test_select_lattice_ties(dev):
    """Integer lattice: many equal distances, ties broken by index."""
    check_self(dev, edge_clouds_for_knn(2, 1024, seed=5), 32)


def test_select_heavy_duplicates_fallback(dev):
    """200 copies of one point: more than the collection capacity lands in one
    bin, so those query blocks take the exact insertion fallback."""
    xyz, _, _ = gaussian_clouds(2, 1024, seed=31)
    xyz[:, :, 100:300] = xyz[:, :, 100:101]
    check_self(dev, xyz, 32)


def test_select_fewer_points_than_k(dev):
    """n < k: unfilled slots stay (10000, 0)."""
    xyz, _, _ = gaussian_clouds(2, 20, seed=3)
    check_self(dev, xyz, 32)


def test_select_far_points_unfilled(dev):
    """Squared distances beyond 10000 are never selected (knn.cu:33-45):
    a cloud of two far-apart clusters leaves slots unfilled."""
    rng = np.random.default_rng(7)
    xyz = rng.standard_normal((2, 3, 1024)).astype(np.float32)
    xyz[:, :, 1000:] += np.float32(500.0)  # 24 points far away: their lists stay short
    check_self(dev, xyz, 32)


def test_select_nan_points(dev):
    """A NaN point never enters any list; its own list stays unfilled."""
    xyz, _, _ = gaussian_clouds(2, 1024, seed=9)
    xyz[0, :, 17] = np.nan
    xyz[1, 1, 400] = np.nan
    check_self(dev, xyz, 32)


@pytest.mark.parametrize("n", [1536, 2048])
def test_select_sorted_2k_edge_cases(dev, n):
    """The extractor's selection at c3 sizes (1024 < n <= 2048) on the inputs
    that exercise its bound growth, tie and fallback paths: a lattice (equal
    distances), 300 copies of one point, far points past 10000, NaN points,
    an outlier facing the cloud; k = 32, 16, 1."""
    xyz = np.concatenate([edge_clouds_for_knn(1, n, seed=11),
                          gaussian_clouds(3, n, seed=n + 3)[0]]).astype(np.float32)
    xyz[1, :, 100:400] = xyz[1, :, 100:101]
    xyz[2, :, n - 40:] += np.float32(500.0)
    xyz[2, :, 3] = np.nan
    xyz[3, 1, 900] = np.nan
    xyz[3, :, 5] = (30.0, 0.0, 0.0)
    xyz = np.ascontiguousarray(xyz)
    nrm = np.ascontiguousarray(np.roll(xyz, 1, axis=1))
    for k in (32, 16, 1):
        _, ei = oracle.knn_dir(xyz, xyz, k)
        check_sorted(dev, xyz, nrm, k, ei)


def test_select_two_sets(dev):
    """Non-self query/candidate sets of different sizes, both directions."""
    from pcr_amd import ops
    rng = np.random.default_rng(11)
    x1 = rng.standard_normal((2, 3, 1024)).astype(np.float32)
    x2 = (rng.standard_normal((2, 3, 900)) * 0.5 + 0.3).astype(np.float32)
    got = ops.knn_forward_cuda(T(x1, dev), T(x2, dev), 32)
    for a, b in zip(got, oracle.knn_forward(x1, x2, 32)):
        assert np.array_equal(N(a), b)


@pytest.mark.parametrize("b,n,k,kind", [(4, 1024, 32, "gauss"), (2, 2048, 32, "gauss"),
                                        (2, 1000, 16, "gauss"), (2, 1024, 32, "edge"),
                                        (2, 1024, 48, "gauss"), (1, 3000, 32, "gauss")])
def test_select_ppf_sorted_emit(dev, b, n, k, kind):
    """pcr_knn_select_ppf (the extractor's selection + PPF): the selection
    writes its ids in sorted query order and the PPF launch un-permutes them
    into knn_idx (k <= 32, n <= 2048); the other shapes take the two-call
    path.  Both bit-exact vs the oracle; every output poisoned first."""
    import torch
    from pcr_amd import _lib
    from pcr_amd.ops import _ptr, _stream
    if kind == "edge":
        xyz = edge_clouds_for_knn(b, n)
    else:
        xyz, _, _ = gaussian_clouds(b, n, seed=n + k)
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    nrm = np.ascontiguousarray(np.roll(xyz, 1, axis=1))
    tx, tn = T(xyz, dev), T(nrm, dev)
    lib = _lib.load()
    ws = torch.full((lib.pcr_knn_workspace_size(b, n, n),), 0xA5, dtype=torch.uint8, device=dev)
    idx = torch.full((b, k, n), -7, dtype=torch.int32, device=dev)
    ppf = torch.full((b, 4, k, n), float("nan"), device=dev)
    _lib.check(lib.pcr_knn_prepare(_ptr(tx), b, n, _ptr(ws), ws.numel(), _stream()), "prepare")
    _lib.check(lib.pcr_knn_select_ppf(_ptr(tx), _ptr(tn), b, n, k, 1, _ptr(idx), _ptr(ppf),
                                      _ptr(ws), ws.numel(), _stream()), "select_ppf")
    torch.cuda.synchronize()
    _, ei = oracle.knn_dir(xyz, xyz, k)
    assert np.array_equal(N(idx), ei)
    ep = oracle.local_ppf(xyz, nrm, xyz, nrm, ei, kmajor=True, relative=True)
    assert np.array_equal(N(ppf), ep, equal_nan=True)
