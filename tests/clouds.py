"""Seeded synthetic point clouds for parity tests, fixtures and the bench
(xyz ~ N(0, I3), unit normals, features ~ U(-1, 1))."""
import numpy as np


def gaussian_clouds(b, n, seed=0, c=0):
    rng = np.random.default_rng(seed)
    xyz = rng.standard_normal((b, 3, n)).astype(np.float32)
    xyz -= xyz.mean(axis=2, keepdims=True)
    nrm = rng.standard_normal((b, 3, n)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    feat = rng.uniform(-1, 1, (b, c, n)).astype(np.float32) if c else None
    return xyz, nrm.astype(np.float32), feat


def edge_norm_coords(n_random, seed=1):
    """Normalised coords [3, n] with the spherical-voxel edge cases first:
    +x axis (known answer), x == 0 with y != 0 and y == 0, north / south
    pole (south is dropped: beta == float(pi) >= PI), centroid (gamma == 0,
    dropped), gamma == 1 (dropped), a duplicate pair, x < 0 on the y == 0
    plane, and then random points inside the unit ball."""
    pts = [
        (0.5, 0.0, 0.0),     # KAT: r=16 -> gx 8, gy 0, gz 8 -> ind 2056
        (0.0, 0.5, 0.0),     # x == 0, y > 0 -> alpha = pi/2 + pi/r
        (0.0, -0.5, 0.0),    # x == 0, y < 0 -> alpha = -pi/2 + pi/r + 2 pi
        (0.0, 0.0, 0.5),     # north pole, x == y == 0 -> alpha = pi/r
        (0.0, 0.0, -0.5),    # south pole -> dropped
        (0.0, 0.0, 0.0),     # centroid -> dropped
        (1.0, 0.0, 0.0),     # gamma == 1 -> dropped
        (0.6, 0.8, 0.0),     # gamma rounds to 1 -> dropped
        (-0.3, 0.0, 0.1),    # x < 0, y == 0 -> alpha = pi + pi/r
        (0.25, -0.25, 0.3),
        (0.25, -0.25, 0.3),  # duplicate
        (-0.0, 0.7, -0.2),   # negative zero x
        (0.999, 0.0, 0.0),
        (1e-30, 1e-30, 1e-30),
    ]
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((n_random, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v *= rng.uniform(0.0, 0.999, (n_random, 1)) ** (1.0 / 3.0)
    allp = np.concatenate([np.array(pts, dtype=np.float64), v], axis=0)
    return np.ascontiguousarray(allp.T.astype(np.float32))


def edge_clouds_for_knn(b, n, seed=2):
    """Clouds with exact duplicates and equidistant points (tie-breaking)."""
    rng = np.random.default_rng(seed)
    xyz = rng.integers(-4, 5, size=(b, 3, n)).astype(np.float32) * 0.25  # lattice -> many ties
    d = min(8, n - n // 2)
    xyz[:, :, n // 2:n // 2 + d] = xyz[:, :, 0:d]  # duplicates
    return np.ascontiguousarray(xyz)
