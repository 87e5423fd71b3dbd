"""Oracle of the feature-space mutual-NN matching (SURVEY.md 8f row f1,
datasets/deepgmr_mn40.py:232-244) against the reference's own numpy
expression, and known answers.  CPU only.

The reference evaluates diff with numpy float32 (BLAS-order channel sums);
the oracle (and the GPU kernel, bit for bit) uses k-ordered fmaf chains.
Argmins therefore agree except where two candidates are within a few fp32
ulps of diff: such near-ties are excluded from the comparison (parity
unpinned there -- the reference's own result depends on its BLAS)."""
import numpy as np
import pytest

import oracle


def numpy_reference(a, b):
    """The reference's expression (deepgmr_mn40.py:235-243), float32."""
    diff = np.power(np.linalg.norm(a, axis=1, keepdims=True), 2) + \
        np.power(np.linalg.norm(b, axis=1, keepdims=True).T, 2) - 2 * np.dot(a, b.T)
    c12 = np.argmin(diff, axis=1)
    c21 = np.argmin(diff, axis=0)
    mask = c21[c12] == np.arange(c12.shape[0])
    return diff, c12, c21, np.arange(c12.shape[0])[mask], c12[mask]


def _clear(diff, axis, tol):
    """Rows (axis=1) / columns (axis=0) whose best and second-best diff differ
    by more than tol (relative to the magnitudes involved)."""
    s = np.sort(diff, axis=axis)
    best, second = np.take(s, 0, axis=axis), np.take(s, 1, axis=axis)
    scale = np.abs(diff).max(axis=axis) + 1e-30
    return (second - best) > tol * scale


@pytest.mark.parametrize("p,n1,n2,c", [(2, 300, 280, 64), (1, 257, 513, 33), (1, 128, 128, 512)])
def test_oracle_matches_numpy_reference(p, n1, n2, c):
    rng = np.random.default_rng(n1 + c)
    f1 = rng.standard_normal((p, n1, c), dtype=np.float32)
    f2 = rng.standard_normal((p, n2, c), dtype=np.float32)
    c12, c21, i1, i2, cnt = oracle.mutual_nn(f1, f2)
    for q in range(p):
        diff, r12, r21, ri1, ri2 = numpy_reference(f1[q], f2[q])
        ok_r = _clear(diff, 1, 1e-5)
        ok_c = _clear(diff, 0, 1e-5)
        assert ok_r.mean() > 0.9 and ok_c.mean() > 0.9
        assert np.array_equal(c12[q][ok_r], r12[ok_r])
        assert np.array_equal(c21[q][ok_c], r21[ok_c])
        if ok_r.all() and ok_c.all():
            assert cnt[q] == len(ri1)
            assert np.array_equal(i1[q, :cnt[q]], ri1) and np.array_equal(i2[q, :cnt[q]], ri2)
        assert np.all(i1[q, cnt[q]:] == -1) and np.all(i2[q, cnt[q]:] == -1)


def test_permuted_features_match_their_permutation():
    """feat2 = feat1 permuted (distinct rows): every point's mutual partner
    is itself, so idx2 = perm^-1[idx1] for all n points."""
    rng = np.random.default_rng(7)
    n, c = 200, 16
    f1 = rng.standard_normal((1, n, c), dtype=np.float32)
    perm = rng.permutation(n)
    f2 = f1[:, perm]
    c12, c21, i1, i2, cnt = oracle.mutual_nn(f1, f2)
    inv = np.argsort(perm)
    assert cnt[0] == n
    assert np.array_equal(i1[0], np.arange(n))
    assert np.array_equal(i2[0], inv)


def test_ties_take_the_first_index_and_nan_first():
    """np.argmin semantics: equal diffs -> the lowest index; a NaN diff wins
    (argmin returns the first NaN)."""
    f1 = np.zeros((1, 2, 2), np.float32)
    f1[0, 0] = [1, 0]
    f1[0, 1] = [0, 1]
    f2 = np.zeros((1, 3, 2), np.float32)
    f2[0, 0] = [0, 1]
    f2[0, 1] = [1, 0]
    f2[0, 2] = [1, 0]  # duplicate of row 1: row 0 of f1 ties between 1 and 2
    c12, c21, i1, i2, cnt = oracle.mutual_nn(f1, f2)
    assert list(c12[0]) == [1, 0]
    assert list(c21[0]) == [1, 0, 0]
    assert cnt[0] == 2 and list(i1[0]) == [0, 1] and list(i2[0]) == [1, 0]
    f2[0, 2] = [np.nan, 0]
    c12, c21, _, _, _ = oracle.mutual_nn(f1, f2)
    assert list(c12[0]) == [2, 2]
