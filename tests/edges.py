"""Bin-edge analysis of spherical voxel indices (hard part 1).

The spherical voxel index (spherical_vox.cu:37-65) floors three pre-floor
values: gamma * r, (alpha * r / 2) / PI and (beta * r) / PI.  Two
normalisations of the same cloud that differ by a few ulps (fixed-order fp64
vs torch's fp32 reduction), or the FMA-contracted vs plain distance chain,
can put a point in a different voxel only when one of those values lies
within a few ulps of an integer (or gamma of the drop edge 1.0).  These
helpers recompute the pre-floor values in float64 and decide, for every
point whose index differs between two variants, whether the difference is
such an edge crossing."""
import numpy as np


def prefloor(nc, r):
    """nc [3, n] normalised coords -> float64 (gamma, gx, gy, gz) pre-floor
    values [4, n] (gamma itself first, for the drop edge)."""
    x, y, z = (nc[i].astype(np.float64) for i in range(3))
    gama = np.sqrt(x * x + y * y + z * z)
    with np.errstate(divide="ignore", invalid="ignore"):
        beta = np.arccos(np.clip(z / gama, -1.0, 1.0))
        alpha = np.where(x == 0, np.where(y == 0, 0.0, np.sign(y) * np.pi * 0.5),
                         np.arctan(y / x) + np.pi * (1.0 - np.sign(x)) / 2.0)
    alpha = alpha + np.pi / r
    alpha = np.where(alpha < 0, alpha + 2 * np.pi, alpha)
    return np.stack([gama, gama * r, alpha * r / 2.0 / np.pi, beta * r / np.pi])


def explain(nc_a, nc_b, ind_a, ind_b, r, ulps=8):
    """For the points of one cloud whose indices differ between variant a
    and b: (count, count explained by a bin-edge crossing, the worst
    unexplained distance to an edge).  An axis whose bin differs is
    explained when both variants' pre-floor values lie within s + |a - b| of
    an integer (s = `ulps` fp32 ulps of the value); a point
    kept by one variant and dropped by the other when gamma is within s of
    1.0 (the gamma >= 1 drop) or the polar value at r (the south-pole drop)."""
    diff = np.nonzero(ind_a != ind_b)[0]
    if diff.size == 0:
        return 0, 0, 0.0
    pa, pb = prefloor(nc_a[:, diff], r), prefloor(nc_b[:, diff], r)
    eps = np.float64(2.0 ** -23)
    ok = np.zeros(diff.size, bool)
    worst = 0.0
    for t in range(diff.size):
        ia, ib = int(ind_a[diff[t]]), int(ind_b[diff[t]])
        if ia < 0 or ib < 0:
            g = np.array([pa[0, t], pb[0, t]])
            zz = np.array([pa[3, t], pb[3, t]])
            s = ulps * eps
            ok[t] = bool(np.any(np.abs(g - 1.0) <= s) or np.any(np.abs(zz - r) <= ulps * eps * r))
            if not ok[t]:
                worst = max(worst, float(np.min(np.abs(g - 1.0))))
            continue
        axes_a = (ia // (r * r), (ia // r) % r, ia % r)
        axes_b = (ib // (r * r), (ib // r) % r, ib % r)
        good = True
        for ax in range(3):
            if axes_a[ax] == axes_b[ax]:
                continue
            va, vb = pa[1 + ax, t], pb[1 + ax, t]
            # both values within a few ulps (plus the variants' own
            # difference) of an integer bin edge (the polar / radial edge 0
            # or r, and the azimuth seam, are integers too)
            tol = ulps * eps * max(abs(va), abs(vb), 1.0) + abs(va - vb)
            da, db = abs(va - np.round(va)), abs(vb - np.round(vb))
            if da > tol or db > tol:
                good = False
                worst = max(worst, float(max(da, db)))
        ok[t] = good
    return int(diff.size), int(ok.sum()), worst
