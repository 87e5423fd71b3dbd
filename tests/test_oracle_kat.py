"""CPU: the oracle against hand-derived known answers, the independent NumPy
restatement and the committed golden fixtures.  (Parity vs genuine reference
output is unpinned: the reference has no fixtures and could not be run.)"""
import os

import numpy as np
import pytest

import oracle
from oracle import np_restate as R
from clouds import gaussian_clouds, edge_norm_coords, edge_clouds_for_knn

GOLDEN = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
PI = np.arccos(-1.0)


def test_kat_positive_x_axis():
    # (0.5, 0, 0), r = 16: gamma 0.5 -> gx 8; alpha = 0 + pi/16 -> gy 0;
    # beta = acosf(0) = float(pi/2) > pi/2 -> beta*16/pi = 8.0000002 -> gz 8
    ind = oracle.sph_index(np.array([[0.5], [0.0], [0.0]], np.float32), 16)
    assert ind[0] == 8 * 256 + 0 * 16 + 8 == 2056


def test_kat_drops():
    pts = np.array([[0, 0, 1, 0.6], [0, 0, 0, 0.8], [-0.5, 0, 0, 0]], np.float32)
    # south pole (beta = float(pi) >= PI), centroid, gamma == 1, gamma ~ 1
    assert (oracle.sph_index(pts, 16) == -1).all()


def test_kat_axis_branches():
    r = 16
    # x == 0, y > 0: alpha = pi/2 + pi/r = 1.7671459 -> gy = floor(1.7671459*16/2/pi) = 4
    # gamma 0.5 -> 8; beta = pi/2 -> gz 8
    assert oracle.sph_index(np.array([[0.0], [0.5], [0.0]], np.float32), r)[0] == 8 * 256 + 4 * 16 + 8
    # north pole x == y == 0: alpha = pi/r -> gy 0; beta = 0 -> gz 0
    assert oracle.sph_index(np.array([[0.0], [0.0], [0.5]], np.float32), r)[0] == 8 * 256
    # x < 0, y == 0: alpha = atan(-0)=-0 + pi + pi/r -> gy = floor(8.5) = 8
    assert oracle.sph_index(np.array([[-0.5], [0.0], [0.0]], np.float32), r)[0] == 8 * 256 + 8 * 16 + 8


def test_kat_global_ppf_self_pair():
    # point == centre: d = 0 -> d_norm = 1e-20f, d/d_norm = 0 -> both angles acos(0)
    p = np.array([[[0.3]], [[0.2]], [[0.1]]], np.float32).reshape(1, 3, 1)
    nrm = np.array([1, 0, 0], np.float32).reshape(1, 3, 1)
    cn = np.array([0, 1, 0], np.float32).reshape(1, 3, 1)
    out = oracle.spherical_ppf_forward(p, p, nrm, cn)[0, :, 0]
    assert out[0] == np.float32(PI / 2) and out[1] == np.float32(PI / 2)
    assert out[2] == np.float32(PI / 2)
    assert out[3] == np.float32(1e-20)


def test_kat_knn_ties_and_fill():
    x1 = np.zeros((1, 3, 1), np.float32)
    x2 = np.array([[[1, -1, 0, 1, 2]], [[0, 0, 0, 0, 0]], [[0, 0, 0, 0, 0]]], np.float32)
    x2 = x2.reshape(1, 3, 5)
    d, i = oracle.knn_dir(x1, x2, 7)
    assert list(i[0, :, 0]) == [2, 0, 1, 3, 4, 0, 0]  # ties keep the lower index
    assert list(d[0, :, 0]) == [0, 1, 1, 1, 4, 10000, 10000]


def test_kat_devox_quirk():
    # integer-division gama_lo = 0 and radian fractions: every corner lies in
    # [0, r^2 + 8r + 5)
    r = 16
    nc = edge_norm_coords(300, seed=9)[None]
    feat = np.ones((1, 1, nc.shape[2]), np.float32)
    _, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    grid = np.zeros((1, 1, r ** 3), np.float32)
    _, inds, _ = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    ok = ind[0] >= 0
    assert inds[0][:, ok].max() < r * r + 8 * r + 5
    assert (inds[0][0, ~ok] == -1).all()


def test_oracle_vs_numpy_restatement_random():
    xyz, nrm, feat = gaussian_clouds(2, 700, seed=21, c=3)
    nc = oracle.normalize_sph(xyz)
    for r in (7, 16, 32):
        a = oracle.spherical_avg_voxelize_forward(feat, nc, r)
        b = R.sph_vox(feat, nc, r)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        grid = np.random.default_rng(r).standard_normal((2, 3, r ** 3)).astype(np.float32)
        a = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, b[1])
        b2 = R.sph_devox(r, nc, grid, b[1])
        assert all(np.array_equal(x, y) for x, y in zip(a, b2))
    x = edge_clouds_for_knn(1, 120, seed=3)
    for k in (1, 5, 33):
        a = oracle.knn_dir(x, x, k)
        b = R.knn_dir(x, x, k)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_golden_fixtures_reproduce():
    g = GOLDEN
    out, ind, cnt = oracle.spherical_avg_voxelize_forward(g["svox_feat"], g["svox_coords"],
                                                          int(g["svox_r"]))
    assert np.array_equal(out, g["svox_out"]) and np.array_equal(ind, g["svox_ind"])
    assert np.array_equal(cnt, g["svox_cnt"])
    d1, d2, i1, i2 = oracle.knn_forward(g["knn_x1"], g["knn_x2"], int(g["knn_k"]))
    assert np.array_equal(i1, g["knn_i1"]) and np.array_equal(i2, g["knn_i2"])
    assert np.array_equal(oracle.ball_query(g["bq_pts"], g["bq_pts"], 0.3, 32), g["bq_idx"])
    assert np.array_equal(oracle.normalize_sph(g["norm_in"]), g["norm_out"])


def test_normalize_close_to_torch_semantics():
    torch = pytest.importorskip("torch")
    xyz, _, _ = gaussian_clouds(3, 1000, seed=4)
    xyz = xyz * np.float32(3.0) + np.float32(1.0)
    t = torch.from_numpy(xyz)
    c = t - t.mean(2, keepdim=True)
    ref = (c / (c.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values + 1e-20)).numpy()
    assert np.abs(oracle.normalize_sph(xyz) - ref).max() < 1e-6


def test_local_ppf_close_to_torch_model_block():
    torch = pytest.importorskip("torch")
    xyz, nrm, _ = gaussian_clouds(1, 300, seed=6)
    xyz = xyz * np.float32(0.4)
    idx = oracle.ball_query(xyz, xyz, 0.3, 16)
    lp = oracle.local_ppf(xyz, nrm, xyz, nrm, idx, kmajor=False, relative=True)
    tx, tn = torch.from_numpy(xyz), torch.from_numpy(nrm)
    ti = torch.from_numpy(idx).long()  # [b, m, u]
    gx = torch.stack([tx[0][:, ti[0]]])  # [1, 3, m, u]
    gn = torch.stack([tn[0][:, ti[0]]])
    rel = (gx - tx.unsqueeze(-1)).permute(0, 1, 3, 2)  # BallQuery output [b,3,u,m]
    nb = gn.permute(0, 1, 3, 2)
    d = tx.unsqueeze(2) - rel
    dn = torch.norm(d, dim=1, keepdim=True)
    du = d / dn
    c = tn.unsqueeze(2).expand_as(nb)
    cos = torch.cat(((nb * du).sum(1, keepdim=True), (c * du).sum(1, keepdim=True),
                     (nb * c).sum(1, keepdim=True)), 1).clamp(-1, 1).numpy()
    assert np.abs(np.cos(lp[:, :3]) - cos).max() < 2e-6
    assert np.abs(lp[:, 3:] - dn.numpy()).max() < 1e-6


def test_acosf_fast_faithful():
    """The local PPF's fp32 acos (pcr_acosf_fast) against float64 arccos:
    <= 1.2 ulp everywhere on [-1, 1] (dense sweep + both range seams), exact
    at -1, 0, 1, NaN in -> NaN out."""
    rng = np.random.default_rng(0)
    step = np.float32(6e-8)
    x = np.concatenate([np.linspace(-1, 1, 400_001, dtype=np.float32),
                        rng.uniform(-1, 1, 400_000).astype(np.float32),
                        np.float32(0.5) + np.arange(-2000, 2000, dtype=np.float32) * step,
                        np.float32(-0.5) + np.arange(-2000, 2000, dtype=np.float32) * step,
                        np.float32(1) - np.arange(0, 20000, dtype=np.float32) * step,
                        np.float32(-1) + np.arange(0, 20000, dtype=np.float32) * step])
    x = np.clip(x, -1, 1).astype(np.float32)
    y = oracle.acosf_fast(x).astype(np.float64)
    ref = np.arccos(x.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert (np.abs(y - ref) / ulp).max() <= 1.2
    e = oracle.acosf_fast(np.array([-1, 0, 1, np.nan], np.float32))
    assert e[0] == np.float32(np.pi) and e[1] == np.float32(np.pi / 2) and e[2] == 0
    assert np.isnan(e[3])
