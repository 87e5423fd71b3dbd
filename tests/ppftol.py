"""Tolerance of the local PPF (pvcnn_classify.py:258-269) for a kernel whose
unit vector comes from the hardware reciprocal square root (v_rsq_f32,
~1 ulp) instead of IEEE divisions, against the oracle's restatement.

The north-star tolerance is 1e-5 on the angles.  acos is ill-conditioned at
+-1: a dot product that differs by a few ulps moves acos(x) near x = +-1 by
up to sqrt(2 |dx|) (3.5e-4 for |dx| = 6e-8), more than 1e-5 -- for any two
implementations that are not bit-identical, the reference itself included
(torch.acos of torch's own sums).  So each angle's bound is 1e-5 plus the
change of acos over the dot products within `eps_dot` of the oracle's:

    |got - exp| <= 1e-5 + max(|acos(c - eps) - exp|, |acos(c + eps) - exp|),
    c = cos(exp)

eps_dot = 1e-6 covers a unit vector within 3 ulps per component (|n| = 1):
|d(n . u)| <= |n| |du| + 3 roundings.  The fourth channel, |d|, is within
2 ulps relative (v_sqrt_f32).  NaN where the oracle has NaN (zero offsets)."""
import numpy as np


def ppf_bound(exp, eps_dot=1e-6, tol=1e-5):
    exp = np.asarray(exp, np.float64)
    ang = exp[..., :3, :, :]
    c = np.cos(ang)
    lo = np.arccos(np.clip(c - eps_dot, -1.0, 1.0))
    hi = np.arccos(np.clip(c + eps_dot, -1.0, 1.0))
    cond = np.maximum(np.abs(lo - ang), np.abs(hi - ang))
    b = np.empty_like(exp)
    b[..., :3, :, :] = tol + cond
    b[..., 3, :, :] = 2.5e-7 * np.abs(exp[..., 3, :, :]) + 1e-30
    return b


def assert_ppf_close(got, exp, eps_dot=1e-6):
    """Local PPF [.., 4, u, n] within ppf_bound of the oracle; returns the
    worst angle difference and how many elements needed more than 1e-5."""
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    nan_e, nan_g = np.isnan(exp), np.isnan(got)
    assert np.array_equal(nan_e, nan_g), "NaN pattern differs"
    b = ppf_bound(np.where(nan_e, 0.0, exp), eps_dot)
    d = np.abs(np.where(nan_e, 0.0, got - exp))
    bad = d > b
    assert not bad.any(), "%d elements outside the bound; worst excess %.3g" % (
        int(bad.sum()), float((d - b).max()))
    ang = d[..., :3, :, :]
    return float(ang.max()), int((ang > 1e-5).sum())
