"""Independent NumPy restatement of the reference kernels (test infrastructure).

Written separately from ``pcr_oracle.c`` (different algorithms where possible:
sort-based top-k instead of insertion, ``np.add.at`` scatter, vectorised
corner maths, NumPy's own float64 ``arccos``/``arctan`` rounded to float32)
so that a restatement bug in either shows up as a disagreement.  Small inputs
only.  Citations are relative to the reference's PVCNN/modules/functional/src.
"""
import numpy as np

PI = np.float64(np.arccos(-1.0))
F32 = np.float32
F64 = np.float64
LD = np.longdouble


def fmaf(a, b, c):
    """float32 fused multiply-add emulated in 80-bit long double."""
    return (LD(1) * np.asarray(a, F32).astype(LD) * np.asarray(b, F32).astype(LD)
            + np.asarray(c, F32).astype(LD)).astype(F32)


def sumsq3(x, y, z):
    return fmaf(z, z, fmaf(x, x, (np.asarray(y, F32) * np.asarray(y, F32)).astype(F32)))


def f2i(v):
    v = np.asarray(v, dtype=F64)
    out = np.zeros(v.shape, np.int64)
    ok = ~np.isnan(v)
    out[ok] = np.trunc(np.clip(v[ok], -2.0 ** 31, 2.0 ** 31 - 1)).astype(np.int64)
    return out.astype(np.int32)


# ------------------------------------------------- spherical coordinates
def sph_coords(x, y, z, r):
    """spherical_vox.cu:34-56 vectorised; returns (valid, gama, alpha, beta)."""
    x, y, z = (np.asarray(v, F32) for v in (x, y, z))
    with np.errstate(all="ignore"):
        gama = np.sqrt(sumsq3(x, y, z)).astype(F32)
        zg = (z / gama).astype(F32)
        valid = ~((gama == 0) | (gama >= 1) | (zg > 1) | (zg < -1))
        beta = np.arccos(zg.astype(F64)).astype(F32)
        valid &= ~(beta.astype(F64) >= PI)
        sgn_y = (y / np.abs(y)).astype(F32)
        sgn_x = (x / np.abs(x)).astype(F32)
        a_axis = (sgn_y.astype(F64) * PI * 0.5).astype(F32)
        at = np.arctan((y / x).astype(F32).astype(F64)).astype(F32)
        a_gen = (at.astype(F64) + PI * (F32(1) - sgn_x).astype(F64) / 2.0).astype(F32)
        alpha = np.where((x == 0) & (y != 0), a_axis, np.where((x == 0) & (y == 0), F32(0), a_gen))
        alpha = (alpha.astype(F64) + PI / F64(r)).astype(F32)
        alpha = np.where(alpha < 0, (alpha.astype(F64) + 2.0 * PI).astype(F32), alpha)
    return valid, gama, alpha, beta


def sph_index(x, y, z, r):
    valid, gama, alpha, beta = sph_coords(x, y, z, r)
    with np.errstate(all="ignore"):
        gx = f2i(np.floor((gama * F32(r)).astype(F32)))
        gy = f2i(np.floor(((alpha * F32(r)).astype(F32) / F32(2)).astype(F32).astype(F64) / PI))
        gz = f2i(np.floor((beta * F32(r)).astype(F32).astype(F64) / PI))
    gx = np.minimum(gx, r - 1)
    gy = np.minimum(gy, r - 1)
    gz = np.minimum(gz, r - 1)
    ind = (gx * r * r + gy * r + gz).astype(np.int32)
    return np.where(valid, ind, -1).astype(np.int32)


def inv_count(cnt):
    return (1.0 / np.asarray(cnt, F32).astype(F64)).astype(F32)


def sph_vox(features, coords, r):
    features = np.asarray(features, F32)
    b, c, n = features.shape
    r3 = r ** 3
    out = np.zeros((b, c, r3), F32)
    ind = np.zeros((b, n), np.int32)
    cnt = np.zeros((b, r3), np.int32)
    for bi in range(b):
        ind[bi] = sph_index(coords[bi, 0], coords[bi, 1], coords[bi, 2], r)
        v = ind[bi] >= 0
        cnt[bi] = np.bincount(ind[bi][v], minlength=r3)
        pts = np.nonzero(v)[0]
        inv = inv_count(cnt[bi][ind[bi][pts]])
        for j in range(c):
            np.add.at(out[bi, j], ind[bi][pts], (features[bi, j, pts] * inv).astype(F32))
    return out, ind, cnt


def sph_devox(r, coords, feat, g_inds):
    """spherical_trilinear_devox.cu:41-135 vectorised over points."""
    feat = np.asarray(feat, F32)
    b, c = feat.shape[:2]
    feat = feat.reshape(b, c, -1)
    n = coords.shape[2]
    r2, r3 = r * r, r ** 3
    inds = np.zeros((b, 8, n), np.int32)
    wgts = np.zeros((b, 8, n), F32)
    outs = np.zeros((b, c, n), F32)
    for bi in range(b):
        pos = g_inds[bi].astype(np.int64)
        valid, gama, alpha, beta = sph_coords(coords[bi, 0], coords[bi, 1], coords[bi, 2], r)
        neg = pos == -1
        inds[bi, 0, neg] = -1
        ok = valid & ~neg
        gg = pos // r2
        ga = (pos - gg * r2) // r
        gb = pos - gg * r2 - ga * r
        glo = (gg // r).astype(F32)
        alo = (PI * 2 * ga / r).astype(F32)
        blo = (PI * gb / r).astype(F32)
        gd1, ad1, bd1 = (gama - glo).astype(F32), (alpha - alo).astype(F32), (beta - blo).astype(F32)
        gd0, ad0, bd0 = (F32(1) - gd1), (F32(1) - ad1), (F32(1) - bd1)
        w = [gd0 * ad0 * bd0, gd0 * ad0 * bd1, gd0 * ad1 * bd0, gd0 * ad1 * bd1,
             gd1 * ad0 * bd0, gd1 * ad0 * bd1, gd1 * ad1 * bd0, gd1 * ad1 * bd1]
        gl, al, bl = f2i(glo), f2i(alo), f2i(blo)
        gh = np.where(gd1 > 0, -1, 0)
        ah = np.where(ad1 > 0, -1, 0)
        bh = np.where(bd1 > 0, 1, 0)
        i0 = gl * r2 + al * r + bl
        i1 = i0 + bh
        i2 = i0 + (ah & r)
        i3 = i2 + bh
        i4 = i0 + (gh & r2)
        i5 = i4 + bh
        i6 = i4 + (ah & r)
        i7 = i6 + bh
        idx = [i0, i1, i2, i3, i4, i5, i6, i7]
        for q in range(8):
            inds[bi, q, ok] = idx[q][ok]
            wgts[bi, q, ok] = w[q][ok]
        pts = np.nonzero(ok)[0]
        for j in range(c):
            fv = [np.where((idx[q][pts] >= 0) & (idx[q][pts] < r3),
                           feat[bi, j, np.clip(idx[q][pts], 0, r3 - 1)], F32(0)) for q in range(8)]
            acc = (w[1][pts] * fv[1]).astype(F32)
            acc = fmaf(w[0][pts], fv[0], acc)
            for q in range(2, 8):
                acc = fmaf(w[q][pts], fv[q], acc)
            outs[bi, j, pts] = acc
    return outs, inds, wgts


# ----------------------------------------------------------------- KNN
def knn_dir(xyz1, xyz2, k):
    """KnnKernel (knn.cu:5-49) as a lexicographic (dist, j) sort."""
    xyz1, xyz2 = np.asarray(xyz1, F32), np.asarray(xyz2, F32)
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    dist = np.full((b, k, n), F32(10000.0))
    idx = np.zeros((b, k, n), np.int32)
    for bi in range(b):
        t = (xyz1[bi][:, :, None] - xyz2[bi][:, None, :]).astype(F32)  # [c, n, m]
        d = (t[0] * t[0]).astype(F32)
        for p in range(1, c):
            d = fmaf(t[p], t[p], d)
        for i in range(n):
            row = d[i]
            j = np.arange(m)
            keep = row < F32(10000.0)
            order = np.lexsort((j[keep], row[keep]))[:k]
            sel = j[keep][order]
            dist[bi, :len(sel), i] = row[sel]
            idx[bi, :len(sel), i] = sel
    return dist, idx


# ------------------------------------------------------------ ball query
def ball_query(centers, points, radius, u):
    centers, points = np.asarray(centers, F32), np.asarray(points, F32)
    b, _, m = centers.shape
    r2 = F32(radius) * F32(radius)
    idx = np.zeros((b, m, u), np.int32)
    for bi in range(b):
        d = (centers[bi][:, :, None] - points[bi][:, None, :]).astype(F32)
        d2 = fmaf(d[2], d[2], fmaf(d[0], d[0], (d[1] * d[1]).astype(F32)))
        acc = (d2 < r2) & (d2.astype(F64) > 1e-5)
        for j in range(m):
            hits = np.nonzero(acc[j])[0][:u]
            if len(hits):
                idx[bi, j, :] = hits[0]
                idx[bi, j, :len(hits)] = hits
    return idx


# ------------------------------------------------------------------ PPF
def _acos_f64(v):
    return np.arccos(v.astype(F64)).astype(F32)


def global_ppf(coords, center, normals, cnormals):
    """ppf.cu:37-90 vectorised."""
    P, C, Nn, Cn = (np.asarray(a, F32) for a in (coords, center, normals, cnormals))
    with np.errstate(all="ignore"):
        d = (C - P).astype(F32)
        s = np.sqrt(sumsq3(d[:, 0], d[:, 1], d[:, 2])).astype(F32)
        dn = np.where(np.isnan(s), F32(1e-20), np.maximum(s.astype(F64), 1e-20).astype(F32)).astype(F32)
        d = (d / dn[:, None]).astype(F32)
        n1 = np.sqrt(sumsq3(Cn[:, 0], Cn[:, 1], Cn[:, 2])).astype(F32)
        n2 = np.sqrt(sumsq3(Nn[:, 0], Nn[:, 1], Nn[:, 2])).astype(F32)
        bad = (n2.astype(F64) <= 1e-10) | (n1.astype(F64) <= 1e-10)
        cn = (Cn / n1[:, None]).astype(F32)
        nn = (Nn / n2[:, None]).astype(F32)

        def dot(a, b_):
            return fmaf(a[:, 2], b_[:, 2], fmaf(a[:, 0], b_[:, 0], (a[:, 1] * b_[:, 1]).astype(F32)))

        def ang(v):
            v64 = v.astype(F64)
            v64 = np.where(np.isnan(v64), 1.0, np.clip(v64, -1.0, 1.0))
            return np.arccos(v64).astype(F32)

        out = np.stack([ang(dot(d, cn)), ang(dot(d, nn)), ang(dot(cn, nn)), dn], axis=1)
    out[np.broadcast_to(bad[:, None, :], out.shape)] = 0
    return out.astype(F32)


def local_ppf(points, normals, centers, cnormals, idx, kmajor, relative=True):
    """pvcnn_classify.py:258-269 with an explicit neighbour index."""
    P, Nn, C, Cn = (np.asarray(a, F32) for a in (points, normals, centers, cnormals))
    b, _, n = P.shape
    m = C.shape[2]
    idx = np.asarray(idx)
    if not kmajor:
        idx = idx.transpose(0, 2, 1)  # -> [B, U, M]
    u = idx.shape[1]
    out = np.zeros((b, 4, u, m), F32)
    with np.errstate(all="ignore"):
        for bi in range(b):
            s = np.clip(idx[bi], 0, n - 1)
            p = P[bi][:, s]  # [3, U, M]
            pn = Nn[bi][:, s]
            c = np.broadcast_to(C[bi][:, None, :], p.shape)
            cn = np.broadcast_to(Cn[bi][:, None, :], p.shape)
            g = (p - c).astype(F32) if relative else p
            d = (c - g).astype(F32)
            dn = np.sqrt(fmaf(d[2], d[2], fmaf(d[0], d[0], (d[1] * d[1]).astype(F32)))).astype(F32)
            du = (d / dn).astype(F32)

            def dot(a, b_):
                return fmaf(a[2], b_[2], fmaf(a[0], b_[0], (a[1] * b_[1]).astype(F32)))

            out[bi, 0] = _acos_f64(np.clip(dot(pn, du), -1, 1))
            out[bi, 1] = _acos_f64(np.clip(dot(cn, du), -1, 1))
            out[bi, 2] = _acos_f64(np.clip(dot(pn, cn), -1, 1))
            out[bi, 3] = dn
    return out


# -------------------------------------------------------- cube variants
def cube_vox(features, coords, r):
    features = np.asarray(features, F32)
    b, c, n = features.shape
    r3 = r ** 3
    out = np.zeros((b, c, r3), F32)
    ind = (coords[:, 0] * r * r + coords[:, 1] * r + coords[:, 2]).astype(np.int32)
    cnt = np.zeros((b, r3), np.int32)
    for bi in range(b):
        cnt[bi] = np.bincount(ind[bi], minlength=r3)
        inv = inv_count(cnt[bi][ind[bi]])
        for j in range(c):
            np.add.at(out[bi, j], ind[bi], (features[bi, j] * inv).astype(F32))
    return out, ind, cnt


def cube_devox(r, coords, feat):
    feat = np.asarray(feat, F32)
    b, c = feat.shape[:2]
    feat = feat.reshape(b, c, -1)
    x, y, z = (np.asarray(coords[:, a], F32) for a in range(3))
    xl, yl, zl = np.floor(x), np.floor(y), np.floor(z)
    xd1, yd1, zd1 = x - xl, y - yl, z - zl
    xd0, yd0, zd0 = F32(1) - xd1, F32(1) - yd1, F32(1) - zd1
    w = [xd0 * yd0 * zd0, xd0 * yd0 * zd1, xd0 * yd1 * zd0, xd0 * yd1 * zd1,
         xd1 * yd0 * zd0, xd1 * yd0 * zd1, xd1 * yd1 * zd0, xd1 * yd1 * zd1]
    xh = np.where(xd1 > 0, -1, 0)
    yh = np.where(yd1 > 0, -1, 0)
    zh = np.where(zd1 > 0, 1, 0)
    i0 = f2i(xl) * r * r + f2i(yl) * r + f2i(zl)
    i1 = i0 + zh
    i2 = i0 + (yh & r)
    i3 = i2 + zh
    i4 = i0 + (xh & (r * r))
    i5 = i4 + zh
    i6 = i4 + (yh & r)
    i7 = i6 + zh
    idx = [i0, i1, i2, i3, i4, i5, i6, i7]
    inds = np.stack(idx, 1).astype(np.int32)
    wgts = np.stack(w, 1).astype(F32)
    outs = np.zeros((b, c, x.shape[1]), F32)
    for bi in range(b):
        for j in range(c):
            fv = [feat[bi, j, idx[q][bi]] for q in range(8)]
            acc = (w[1][bi] * fv[1]).astype(F32)
            acc = fmaf(w[0][bi], fv[0], acc)
            for q in range(2, 8):
                acc = fmaf(w[q][bi], fv[q], acc)
            outs[bi, j] = acc
    return outs, inds, wgts
