"""GPU parity of the normal estimation kernel (SURVEY.md 8f row f3,
csrc/normals.hip) against the oracle: bit-exact normals and neighbour counts
(both evaluate include/pcr_math.h pcr_estimate_normal in fp64 on the same
neighbour order)."""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds

pytestmark = pytest.mark.gpu


def _sphere(b, n, seed, noise=0.0):
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((b, 3, n))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (0.5 * v + noise * rng.standard_normal((b, 3, n)) + 0.05).astype(np.float32)


@pytest.mark.parametrize("b,n,radius", [(4, 1024, 0.1), (2, 5000, 0.1), (1, 300, 0.3),
                                        (3, 2048, 0.05)])
def test_normals_match_oracle(dev, b, n, radius):
    from pcr_amd import ops
    pts = _sphere(b, n, seed=n, noise=0.01)
    got, cnt = ops.estimate_normals(torch.from_numpy(pts).to(dev), radius, return_counts=True)
    torch.cuda.synchronize()
    en, ec = oracle.estimate_normals(pts, radius)
    assert np.array_equal(cnt.cpu().numpy(), ec)
    assert np.array_equal(got.cpu().numpy(), en)


def test_normals_gaussian_and_get_normals(dev):
    from pcr_amd import io, ops
    xyz, _, _ = gaussian_clouds(2, 1024, seed=4)
    xyz = (xyz * 0.2).astype(np.float32)
    got = ops.estimate_normals(torch.from_numpy(xyz).to(dev), 0.1)
    en, _ = oracle.estimate_normals(xyz, 0.1)
    assert np.array_equal(got.cpu().numpy(), en)
    # the reference's call shape: one [n, 3] numpy cloud -> [n, 3] float32
    one = io.get_normals(np.ascontiguousarray(xyz[0].T))
    assert one.dtype == np.float32 and np.array_equal(one, en[0].T)


@pytest.mark.parametrize("n", [1023, 2049, 7])
def test_normals_ragged_tails(dev, n):
    """Point counts that are not a multiple of 4 run the scalar tail of the
    float4 candidate loop (csrc/normals.hip)."""
    from pcr_amd import ops
    pts = _sphere(2, n, seed=n + 1, noise=0.01)
    got, cnt = ops.estimate_normals(torch.from_numpy(pts).to(dev), 0.1, return_counts=True)
    en, ec = oracle.estimate_normals(pts, 0.1)
    assert np.array_equal(cnt.cpu().numpy(), ec)
    assert np.array_equal(got.cpu().numpy(), en)


def test_normals_radius_boundary(dev):
    """Candidates at |q - p| = radius (1 +- 1e-7) and (1 +- 1e-6) from the
    queries: the fp32 prefilter must pass every candidate the deciding fp64
    radius test accepts, so the counts equal the oracle's exactly."""
    from pcr_amd import ops
    rng = np.random.default_rng(11)
    radius = 0.1
    nq = 40
    q = rng.uniform(-0.5, 0.5, (nq, 3))
    rows = [q]
    for f in (1 - 1e-7, 1 + 1e-7, 1 - 1e-6, 1 + 1e-6, 1.0):
        d = rng.standard_normal((nq, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rows.append(q + radius * f * d)
    pts = np.concatenate(rows + [rng.uniform(-0.5, 0.5, (37, 3))], axis=0)
    pts = np.ascontiguousarray(pts.T[None].astype(np.float32))  # [1, 3, n], n % 4 != 0
    got, cnt = ops.estimate_normals(torch.from_numpy(pts).to(dev), radius, return_counts=True)
    en, ec = oracle.estimate_normals(pts, radius)
    assert np.array_equal(cnt.cpu().numpy(), ec)
    assert np.array_equal(got.cpu().numpy(), en)
