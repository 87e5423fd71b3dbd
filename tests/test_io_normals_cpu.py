"""CPU: SURVEY.md 8f row f3 -- the native ModelNet40 txt parser against
np.loadtxt (bit-exact), the ModelNet40 sample pipeline, and the normal
estimation oracle against numpy's eigensolver.  Open3D is not installed, so
the normals are "parity unpinned" against the reference's get_normals; the
oracle restates Open3D's published algorithm and pins the GPU kernel
(tests/test_gpu_normals.py)."""
import os

import numpy as np
import pytest

import oracle


def _write_cloud(path, rng, n):
    pts = rng.standard_normal((n, 6))
    with open(path, "w") as f:
        for row in pts:
            f.write(",".join("%.6f" % v for v in row) + "\n")
    return pts


def test_txt_parser_matches_loadtxt(tmp_path):
    from pcr_amd import io
    rng = np.random.default_rng(0)
    p = tmp_path / "a.txt"
    _write_cloud(p, rng, 500)
    with open(p, "a") as f:
        f.write("1e-3, -2.5E+01 ,3,4,5,6\r\n\n0.1000000000000000055511151231257827,2,3,4,5,6")
    got = io.read_xyzn_txt(str(p))
    exp = np.loadtxt(str(p), delimiter=",").astype(np.float32)
    assert got.dtype == np.float32 and np.array_equal(got, exp)


def test_txt_parser_errors(tmp_path):
    from pcr_amd import io
    p = tmp_path / "bad.txt"
    p.write_text("1,2,3\n4,5\n")
    with pytest.raises(RuntimeError, match="columns"):
        io.read_xyzn_txt(str(p))
    p.write_text("1,2,x\n")
    with pytest.raises(RuntimeError, match="not a number"):
        io.read_xyzn_txt(str(p))
    with pytest.raises(RuntimeError, match="cannot open"):
        io.read_xyzn_txt(str(tmp_path / "missing.txt"))


def test_modelnet40_dataset(tmp_path):
    from pcr_amd import io
    rng = np.random.default_rng(1)
    for cls in ("airplane", "chair"):
        os.makedirs(tmp_path / cls)
        for i in (1, 2):
            _write_cloud(tmp_path / cls / ("%s_%04d.txt" % (cls, i)), rng, 300)
    (tmp_path / "modelnet40_shape_names.txt").write_text("chair\nairplane\n")
    (tmp_path / "modelnet40_test.txt").write_text("chair_0002\nairplane_0001\n")
    ds = io.ModelNet40Dataset(str(tmp_path), "test", 40, 256)
    assert len(ds) == 2 and ds.classes == ["airplane", "chair"]
    np.random.seed(5)
    pcd, target = ds[0]
    assert target == 1 and pcd.shape == (6, 256) and pcd.dtype == np.float32
    # the reference pipeline, restated with numpy on the same RNG stream
    np.random.seed(5)
    raw = np.loadtxt(str(tmp_path / "chair" / "chair_0002.txt"), delimiter=",")
    idx = np.random.choice(300, 256, replace=False)
    pts = raw[idx, :3].astype(np.float32)
    pts -= np.mean(pts, axis=0, keepdims=True)
    assert np.array_equal(pcd[:3], pts.T)
    assert np.array_equal(pcd[3:], raw[idx, 3:].astype(np.float32).T)
    # random_rot reseeds with 0 each call: the same rotation for every sample
    t1, a = io.random_rotation(np.eye(3))
    t2, b = io.random_rotation(np.eye(3))
    assert np.array_equal(t1, t2) and np.allclose(t1[:3, :3] @ t1[:3, :3].T, np.eye(3))


def test_normals_oracle_against_eigh():
    """Smooth surface: every normal is numpy's smallest eigenvector of the
    same covariance up to sign, oriented towards the origin, unit length."""
    rng = np.random.default_rng(2)
    v = rng.standard_normal((3, 3000))
    v /= np.linalg.norm(v, axis=0)
    pts = (0.6 * v).astype(np.float32)[None]
    nrm, cnt = oracle.estimate_normals(pts, 0.1)
    P = pts[0].astype(np.float64)
    checked = 0
    for j in range(0, 3000, 37):
        d2 = ((P - P[:, j:j + 1]) ** 2).sum(0)
        nb = P[:, d2 < 0.01]
        assert nb.shape[1] == cnt[0, j]
        if nb.shape[1] < 3:
            continue
        w, e = np.linalg.eigh(np.cov(nb, bias=True))
        ref = e[:, 0]
        assert abs(abs(ref @ nrm[0, :, j]) - 1) < 1e-4
        checked += 1
    assert checked > 50
    assert (np.einsum("in,in->n", nrm[0], -P) >= 0).all()        # faces the origin
    assert np.allclose(np.linalg.norm(nrm[0], axis=0), 1, atol=1e-6)
    assert (np.abs(np.einsum("in,in->n", nrm[0], v)) > 0.99).all()  # radial on a sphere


def test_normals_oracle_degenerate_cases():
    # isolated points (< 3 neighbours) -> (0, 0, 1); a flat patch -> the plane
    # normal via the diagonal branch; collinear points stay finite
    iso = np.array([[[0.0, 1.0, 2.0], [0.0, 0.0, 0.0], [1.0, 1.0, 1.0]]], np.float32)
    n, c = oracle.estimate_normals(iso, 0.1)
    assert (c == 1).all() and np.array_equal(n[0].T, np.tile([0, 0, 1], (3, 1)))
    g = np.arange(25)
    flat = np.stack([(g % 5) * 0.02, (g // 5) * 0.02, np.full(25, 0.3)]).astype(np.float32)[None]
    n, c = oracle.estimate_normals(flat, 0.05)
    assert np.allclose(np.abs(n[0, 2]), 1) and (n[0, 2] < 0).all()  # faces the origin (below)
    line = np.stack([np.linspace(0, 0.1, 30), np.zeros(30), np.zeros(30)]).astype(np.float32)[None]
    n, _ = oracle.estimate_normals(line, 0.05)
    assert np.isfinite(n).all() and np.allclose(np.linalg.norm(n[0], axis=0), 1, atol=1e-6)
