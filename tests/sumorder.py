"""fp32 summation-order tolerance for the scatter-add backward passes.

The reference's backward kernels (trilinear_devox.cu:120-163,
spherical_trilinear_devox.cu:150-194, knn.cu:52-78, grouping.cu:55-85)
accumulate with atomicAdd, i.e. in an arbitrary order; the MI355X kernels
sum in their own order and the oracle in ascending point order.  For a sum
of m fp32 products t_i (each product rounded once, as the reference's
`w * g`), any two summation orders differ by at most

    2 * gamma_(m-1) * sum |t_i|,   gamma_j = j u / (1 - j u),  u = 2^-24

(Higham, Accuracy and Stability of Numerical Algorithms, 4.2).  The bound
is per output element, from that element's own terms -- so it is tight for
short sums and grows only where many points share a voxel.
"""
import numpy as np

U = 2.0 ** -24


def gamma(m):
    m = np.asarray(m, dtype=np.float64)
    return m * U / (1.0 - m * U)


def devox_backward_bound(grad_y, inds, wgts, r3, skip_neg=False):
    """Per-element bound [b, c, r3] for devoxelize backward
    (grad_x[b, j, inds[b, q, i]] += wgts[b, q, i] * grad_y[b, j, i])."""
    grad_y = np.asarray(grad_y, np.float32)
    b, c, n = grad_y.shape
    S = np.zeros((b, c, r3), np.float64)
    M = np.zeros((b, r3), np.int64)
    for bi in range(b):
        skip = (inds[bi, 0] == -1) if skip_neg else np.zeros(n, bool)
        for q in range(8):
            v = inds[bi, q].astype(np.int64)
            ok = (v >= 0) & (v < r3) & ~skip
            t = np.abs((wgts[bi, q][ok][None, :] * grad_y[bi][:, ok]).astype(np.float32))
            np.add.at(S[bi], (slice(None), v[ok]), t.astype(np.float64))
            np.add.at(M[bi], v[ok], 1)
    return 2.0 * gamma(np.maximum(M - 1, 0))[:, None, :] * S


def assert_within_sum_order(got, exp, bound, floor=0.0):
    """|got - exp| <= bound (+ floor for denormal-level noise), elementwise."""
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    diff = np.abs(got - exp)
    excess = diff - (bound + floor)
    worst = np.unravel_index(np.argmax(excess), excess.shape)
    assert excess.max(initial=-1.0) <= 0, (
        "sum-order bound exceeded at %s: |diff| %.3g > bound %.3g"
        % (worst, diff[worst], bound[worst] + floor))


def _bound(S, M):
    return 2.0 * gamma(np.maximum(M - 1, 0)) * S


def knn_backward_bound(x1, x2, gd1, gd2, idx1, idx2):
    """Per-element bounds ([b, c, n], [b, c, m]) for knn_backward_cuda
    (knn.cu:52-78, both launches of knn_grad_kernel): for every (query i,
    slot q) with g = 2 gd[q, i] < 20000 the term t_p = g (x1[p, i] -
    x2[p, id]) is added to grad1[p, i] and subtracted from grad2[p, id]; the
    second launch swaps the roles.  Every output element is a sum of such
    terms in atomic order."""
    x1 = np.asarray(x1, np.float32)
    x2 = np.asarray(x2, np.float32)
    b, c, n = x1.shape
    m = x2.shape[2]
    S1 = np.zeros((b, c, n), np.float64)
    S2 = np.zeros((b, c, m), np.float64)
    M1 = np.zeros((b, 1, n), np.int64)
    M2 = np.zeros((b, 1, m), np.int64)

    def direction(xa, xb, gd, idx, Sa, Sb, Ma, Mb, na):
        for bi in range(b):
            g = (np.asarray(gd[bi], np.float32) * np.float32(2)).astype(np.float32)  # [k, na]
            ok = g < np.float32(20000)
            for q in range(g.shape[0]):
                sel = np.nonzero(ok[q])[0]
                ids = np.asarray(idx[bi, q], np.int64)[sel]
                d = (xa[bi][:, sel] - xb[bi][:, ids]).astype(np.float32)
                t = np.abs((g[q, sel][None, :] * d).astype(np.float32)).astype(np.float64)
                Sa[bi][:, sel] += t
                Ma[bi][0, sel] += 1
                np.add.at(Sb[bi], (slice(None), ids), t)
                np.add.at(Mb[bi][0], ids, 1)

    direction(x1, x2, gd1, idx1, S1, S2, M1, M2, n)
    direction(x2, x1, gd2, idx2, S2, S1, M2, M1, m)
    return _bound(S1, M1), _bound(S2, M2)


def grouping_backward_bound(grad_y, idx, n):
    """Per-element bound [b, c, n] for grouping_backward (grouping.cu:58-77):
    grad_x[c, idx[m, u]] += grad_y[c, m, u]."""
    grad_y = np.asarray(grad_y, np.float32)
    b, c, m, u = grad_y.shape
    S = np.zeros((b, c, n), np.float64)
    M = np.zeros((b, 1, n), np.int64)
    for bi in range(b):
        ids = np.asarray(idx[bi], np.int64).reshape(-1)
        np.add.at(S[bi], (slice(None), ids), np.abs(grad_y[bi].reshape(c, -1)).astype(np.float64))
        np.add.at(M[bi][0], ids, 1)
    return _bound(S, M)
