"""Generate tests/golden/golden.npz -- small parity fixtures.

The reference publishes no golden vectors and could not be built or loaded
here, so these vectors are produced by the CPU oracle
(oracle/pcr_oracle.c, a restatement of the reference .cu text) and are
accepted only if the independent NumPy restatement (oracle/np_restate.py)
reproduces every one of them bit for bit.  Inputs and outputs are stored
together.  Re-run with:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from oracle import np_restate as R  # noqa: E402
from clouds import gaussian_clouds, edge_norm_coords, edge_clouds_for_knn  # noqa: E402


def same(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)


def same_lppf(a, b):
    """Local PPF: the oracle's angles use the faithful fp32 acos of the
    kernels (pcr_acosf_fast, <= 1.15 ulp), the NumPy restatement float64
    arccos rounded once: angles within 2.5e-7, |d| bit-exact."""
    a, b = np.asarray(a), np.asarray(b)
    if not np.array_equal(np.isnan(a), np.isnan(b)):
        return False
    ok = ~np.isnan(a)
    return (np.abs(a[:, :3] - b[:, :3])[ok[:, :3]].max(initial=0) <= 2.5e-7
            and np.array_equal(a[:, 3:], b[:, 3:], equal_nan=True))


def main():
    g = {}
    # ---- spherical voxelization on edge + random normalised coords (r=16, C=4)
    r = 16
    nc = np.stack([edge_norm_coords(242, seed=1), edge_norm_coords(242, seed=5)])  # [2,3,256]
    rng = np.random.default_rng(11)
    feat = rng.uniform(-1, 1, (2, 4, nc.shape[2])).astype(np.float32)
    out, ind, cnt = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    o2, i2, c2 = R.sph_vox(feat, nc, r)
    assert same(out, o2) and same(ind, i2) and same(cnt, c2)
    assert ind[0, 0] == 2056, ind[0, 0]  # hand-derived known answer
    g.update(svox_coords=nc, svox_feat=feat, svox_r=np.int32(r), svox_out=out, svox_ind=ind,
             svox_cnt=cnt)
    # FMA sensitivity flags (oracle-only): points whose bin differs without FMA
    _, ind_nofma, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r, use_fma=False)
    g["svox_fma_sensitive"] = (ind != ind_nofma)
    # ---- spherical devoxelization of a random grid at the produced indices
    grid = rng.standard_normal((2, 4, r ** 3)).astype(np.float32)
    outs, inds, wgts = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    o2, i2, w2 = R.sph_devox(r, nc, grid, ind)
    assert same(outs, o2) and same(inds, i2) and same(wgts, w2)
    g.update(sdevox_grid=grid, sdevox_outs=outs, sdevox_inds=inds, sdevox_wgts=wgts)
    # backward fixtures (oracle order; GPU compares within tolerance)
    gy = rng.standard_normal((2, 4, r ** 3)).astype(np.float32)
    g["svox_grad_y"] = gy
    g["svox_grad_x"] = oracle.avg_voxelize_backward(gy, ind, cnt)
    gd = rng.standard_normal((2, 4, nc.shape[2])).astype(np.float32)
    g["sdevox_grad_y"] = gd
    g["sdevox_grad_x"] = oracle.devoxelize_backward(gd, inds, wgts, r, spherical=True)
    # ---- normalisation (fixed-order double mean)
    xyz, nrm, _ = gaussian_clouds(2, 300, seed=3)
    xyz = xyz * np.float32(2.5) + np.float32(0.75)
    g["norm_in"] = xyz
    g["norm_out"] = oracle.normalize_sph(xyz)
    # ---- KNN both directions, lattice clouds (ties) k=16
    x1 = edge_clouds_for_knn(2, 200, seed=2)
    x2 = edge_clouds_for_knn(2, 150, seed=4)
    d1, d2, i1, i2 = oracle.knn_forward(x1, x2, 16)
    rd1, ri1 = R.knn_dir(x1, x2, 16)
    rd2, ri2 = R.knn_dir(x2, x1, 16)
    assert same(d1, rd1) and same(i1, ri1) and same(d2, rd2) and same(i2, ri2)
    g.update(knn_x1=x1, knn_x2=x2, knn_k=np.int32(16), knn_d1=d1, knn_d2=d2, knn_i1=i1,
             knn_i2=i2)
    # k larger than the candidate count -> (10000, 0) slots
    xs = edge_clouds_for_knn(1, 10, seed=6)
    ds1, ds2, is1, is2 = oracle.knn_forward(xs, xs[:, :, :7].copy(), 12)
    g.update(knn_small_x=xs, knn_small_d1=ds1, knn_small_i1=is1, knn_small_d2=ds2,
             knn_small_i2=is2)
    gd1 = rng.standard_normal(d1.shape).astype(np.float32)
    gd2 = rng.standard_normal(d2.shape).astype(np.float32)
    gd1[0, 3, 5] = 10000.0  # >= 20000 after doubling: skipped (knn.cu:68)
    gg1, gg2 = oracle.knn_backward(x1, x2, gd1, gd2, i1, i2)
    g.update(knn_gd1=gd1, knn_gd2=gd2, knn_g1=gg1, knn_g2=gg2)
    # ---- ball query + grouping on gaussian clouds (radius 0.3 -> use 0.6 here)
    pts, pn, _ = gaussian_clouds(2, 256, seed=7)
    pts = pts * np.float32(0.5)
    bq = oracle.ball_query(pts, pts, 0.3, 32)
    assert same(bq, R.ball_query(pts, pts, 0.3, 32))
    g.update(bq_pts=pts, bq_nrm=pn, bq_idx=bq)
    grp = oracle.grouping_forward(pts, bq)
    g["bq_grouped"] = grp
    gy = rng.standard_normal(grp.shape).astype(np.float32)
    g["grp_grad_y"] = gy
    g["grp_grad_x"] = oracle.grouping_backward(gy, bq, pts.shape[2])
    # ---- local PPF (ball-query layout, model's relative quirk) and KNN layout
    lp = oracle.local_ppf(pts, pn, pts, pn, bq, kmajor=False, relative=True)
    assert same_lppf(lp, R.local_ppf(pts, pn, pts, pn, bq, False, True))
    g["lppf_ball"] = lp
    _, ki = oracle.knn_dir(pts, pts, 16)
    lk = oracle.local_ppf(pts, pn, pts, pn, ki, kmajor=True, relative=True)
    assert same_lppf(lk, R.local_ppf(pts, pn, pts, pn, ki, True, True))
    g.update(lppf_knn_idx=ki, lppf_knn=lk)
    # ---- global PPF with zero normals / coincident centre
    cen = np.repeat(pts.mean(axis=2, keepdims=True), pts.shape[2], axis=2)
    cn = np.repeat(pn.mean(axis=2, keepdims=True), pts.shape[2], axis=2)
    pn0 = pn.copy()
    pn0[:, :, 3] = 0.0
    pts0 = pts.copy()
    pts0[:, :, 4] = cen[:, :, 4]
    gp = oracle.spherical_ppf_forward(pts0, cen, pn0, cn)
    assert same(gp, R.global_ppf(pts0, cen, pn0, cn))
    g.update(gppf_pts=pts0, gppf_cen=cen, gppf_nrm=pn0, gppf_cnrm=cn, gppf_out=gp)
    # ---- cube voxelization / devoxelization (cu-dg; normalize=False path)
    rc = 8
    cc = np.clip((pts + 1) / 2 * rc, 0, rc - 1).astype(np.float32)
    vc = np.round(cc).astype(np.int32)  # numpy round-half-even == torch.round
    cf = rng.uniform(-1, 1, (2, 4, pts.shape[2])).astype(np.float32)
    co, ci, cn_ = oracle.avg_voxelize_forward(cf, vc, rc)
    assert all(same(a, b) for a, b in zip((co, ci, cn_), R.cube_vox(cf, vc, rc)))
    cgrid = rng.standard_normal((2, 4, rc ** 3)).astype(np.float32)
    do, di, dw = oracle.trilinear_devoxelize_forward(rc, cc, cgrid)
    assert all(same(a, b) for a, b in zip((do, di, dw), R.cube_devox(rc, cc, cgrid)))
    g.update(cvox_r=np.int32(rc), cvox_cc=cc, cvox_vc=vc, cvox_feat=cf, cvox_out=co,
             cvox_ind=ci, cvox_cnt=cn_, cdevox_grid=cgrid, cdevox_outs=do, cdevox_inds=di,
             cdevox_wgts=dw)
    gdc = rng.standard_normal((2, 4, pts.shape[2])).astype(np.float32)
    g["cdevox_grad_y"] = gdc
    g["cdevox_grad_x"] = oracle.devoxelize_backward(gdc, di, dw, rc, spherical=False)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **g)
    print("wrote", path, os.path.getsize(path), "bytes,", len(g), "arrays")


if __name__ == "__main__":
    main()
