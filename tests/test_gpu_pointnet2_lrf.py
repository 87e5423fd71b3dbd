"""GPU parity of SURVEY.md 8f rows f2 (LRF change_coords, csrc/lrf.hip) and
f4 (PointNet++ ops, csrc/pointnet2.hip) against the oracle, through the C
ABI: bit-exact for indices, picks, and every output whose oracle order is the
kernel's order; 1e-5 for the atomic scatter backwards."""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("b,n", [(3, 1024), (2, 37), (1, 2048), (4, 8192), (2, 20000), (1, 1)])
def test_lrf_matches_oracle(dev, b, n):
    from pcr_amd import ops
    xyz, _, _ = gaussian_clouds(b, n, seed=n + 1)
    xyz = xyz + np.float32(0.5)
    out, (basis, picks, status) = ops.lrf_change_coords(_t(xyz, dev), check=False,
                                                        return_basis=True)
    torch.cuda.synchronize()
    eo, eb, ep, es = oracle.lrf_change_coords(xyz)
    assert np.array_equal(status.cpu().numpy(), es)
    assert np.array_equal(picks.cpu().numpy(), ep)
    assert np.array_equal(basis.cpu().numpy(), eb)
    assert np.array_equal(out.cpu().numpy(), eo)


def test_lrf_ties_and_asserts(dev):
    from pcr_amd import ops
    # a point-symmetric cloud (p and -p): the mean is exactly 0 and every
    # norm occurs twice, so rank 0 is a tie (the lower index wins) and the
    # mirror of base_x (lambda = -1) must be skipped
    half, _, _ = gaussian_clouds(1, 150, seed=9)
    xyz = np.concatenate([half, -half], axis=2)
    out, (basis, picks, status) = ops.lrf_change_coords(_t(xyz, dev), check=False,
                                                        return_basis=True)
    eo, eb, ep, es = oracle.lrf_change_coords(xyz)
    assert np.array_equal(picks.cpu().numpy(), ep)
    assert ep[0, 0] < 150
    assert np.array_equal(out.cpu().numpy(), eo)
    z = np.zeros((2, 3, 16), np.float32)
    z[1] = np.random.default_rng(0).standard_normal((3, 16))
    with pytest.raises(AssertionError, match="pvcnn_classify.py:159"):
        ops.lrf_change_coords(_t(z, dev))
    t = np.linspace(-1, 1, 33, dtype=np.float32)
    line = np.stack([t, 2 * t, -t])[None]
    with pytest.raises(AssertionError, match="pvcnn_classify.py:169"):
        ops.lrf_change_coords(_t(line, dev))


@pytest.mark.parametrize("b,n,m", [(2, 100, 32), (3, 256, 64), (2, 1024, 512), (1, 4096, 256),
                                   (1, 8192, 128), (2, 10000, 64), (1, 5, 9)])
def test_fps_matches_oracle(dev, b, n, m):
    from pcr_amd import ops
    xyz, _, _ = gaussian_clouds(b, n, seed=b * n + m)
    got = ops.furthest_point_sampling(_t(xyz, dev), m)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), oracle.furthest_point_sampling(xyz, m))


@pytest.mark.parametrize("n", [1100, 9000])
def test_fps_ties(dev, n):
    """Integer lattice (exact distances, many ties) with coinciding points k
    and k + 512: the pick follows the reference's 512-thread reduction."""
    from pcr_amd import ops
    g = np.arange(n)
    xyz = np.stack([g % 11, (g // 11) % 10, g // 110]).astype(np.float32)[None]
    xyz[:, :, 512:] = xyz[:, :, :n - 512]
    xyz = np.concatenate([xyz, xyz[:, [1, 0, 2]]], axis=0)
    got = ops.furthest_point_sampling(_t(xyz, dev), 40)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), oracle.furthest_point_sampling(xyz, 40))


def test_gather_features(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(1)
    f = rng.standard_normal((3, 67, 1024)).astype(np.float32)
    idx = rng.integers(0, 1024, (3, 300)).astype(np.int32)
    out = ops.gather_features_forward(_t(f, dev), _t(idx, dev))
    assert np.array_equal(out.cpu().numpy(), oracle.gather_features_forward(f, idx))
    g = rng.standard_normal((3, 67, 300)).astype(np.float32)
    gx = ops.gather_features_backward(_t(g, dev), _t(idx, dev), 1024)
    assert np.abs(gx.cpu().numpy() - oracle.gather_features_backward(g, idx, 1024)).max() <= 1e-5


@pytest.mark.parametrize("b,c,m,n", [(2, 16, 256, 1024), (1, 3, 3000, 700), (2, 4, 2, 50),
                                     (1, 1, 1, 10), (3, 64, 128, 2048)])
def test_three_nn_interpolate(dev, b, c, m, n):
    from pcr_amd import ops
    rng = np.random.default_rng(m + n)
    pts = rng.standard_normal((b, 3, n)).astype(np.float32)
    ctr = rng.standard_normal((b, 3, m)).astype(np.float32)
    cf = rng.standard_normal((b, c, m)).astype(np.float32)
    out, inds, wgts = ops.three_nearest_neighbors_interpolate_forward(
        _t(pts, dev), _t(ctr, dev), _t(cf, dev))
    eo, ei, ew = oracle.three_nearest_neighbors_interpolate_forward(pts, ctr, cf)
    assert np.array_equal(inds.cpu().numpy(), ei)
    assert np.array_equal(wgts.cpu().numpy(), ew)
    assert np.array_equal(out.cpu().numpy(), eo)
    g = rng.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.three_nearest_neighbors_interpolate_backward(_t(g, dev), inds, wgts, m)
    exp = oracle.three_nearest_neighbors_interpolate_backward(g, ei, ew, m)
    assert np.abs(gx.cpu().numpy() - exp).max() <= 1e-5 * max(1.0, np.abs(exp).max())


def test_functional_autograd(dev):
    import PVCNN.modules.functional as F
    rng = np.random.default_rng(3)
    xyz = _t(rng.standard_normal((2, 3, 512)).astype(np.float32), dev)
    centres = F.furthest_point_sample(xyz, 64)
    idx = oracle.furthest_point_sampling(xyz.cpu().numpy(), 64)
    assert torch.equal(centres.cpu(), torch.gather(xyz.cpu(), 2,
                                                   torch.from_numpy(idx).long()[:, None].expand(-1, 3, -1)))
    feat = _t(rng.standard_normal((2, 8, 64)).astype(np.float32), dev).requires_grad_(True)
    out = F.nearest_neighbor_interpolate(xyz, centres, feat)
    out.square().sum().backward()
    # reference autograd: the same interpolation in torch on the saved inds/wgts
    _, ei, ew = oracle.three_nearest_neighbors_interpolate_forward(
        xyz.cpu().numpy(), centres.cpu().numpy(), feat.detach().cpu().numpy())
    f64 = feat.detach().cpu().double().requires_grad_(True)
    ii = torch.from_numpy(ei).long()
    ref = sum(torch.gather(f64, 2, ii[:, a][:, None].expand(-1, 8, -1)) *
              torch.from_numpy(ew[:, a][:, None]).double() for a in range(3))
    ref.square().sum().backward()
    assert torch.allclose(feat.grad.cpu().double(), f64.grad, atol=1e-4)
    src = _t(rng.standard_normal((2, 5, 512)).astype(np.float32), dev).requires_grad_(True)
    g = F.gather(src, torch.from_numpy(idx).to(dev))
    g.sum().backward()
    cnt = np.zeros((2, 512), np.float32)
    for q in range(2):
        np.add.at(cnt[q], idx[q], 1.0)
    assert np.array_equal(src.grad.cpu().numpy(), np.repeat(cnt[:, None], 5, 1))
