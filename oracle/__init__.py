"""CPU parity oracle for the rotation-invariant-feature hot path.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this package.  The product package never imports it.

PARITY UNPINNED: the reference ships no tests/fixtures/golden vectors and
compiling or loading the reference extension here was denied, so
this restatement (``pcr_oracle.c``, written from the reference's .cu text) is
pinned by an independent NumPy restatement (``np_restate.py``) and by
hand-derived known answers (tests/test_oracle_kat.py), not by reference output.

Every wrapper takes/returns contiguous numpy arrays in the reference layouts
(channel-major ``[B, C, N]`` fp32, int32 indices).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpcr_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i = ctypes.c_int
_f = ctypes.c_float

_SIGS = {
    "orc_knn_dir": [_i, _i, _i, _i, _i, _f32p, _f32p, _f32p, _i32p],
    "orc_knn_grad": [_i, _i, _i, _i, _i, _f32p, _f32p, _f32p, _f32p, _i32p, _i32p, _f32p, _f32p],
    "orc_global_ppf": [_i, _i, _f32p, _f32p, _f32p, _f32p, _f32p],
    "orc_sph_vox": [_i, _i, _i, _i, _f32p, _f32p, _f32p, _i32p, _i32p, _i],
    "orc_avg_vox_grad": [_i, _i, _i, _i, _i32p, _i32p, _f32p, _f32p],
    "orc_sph_devox": [_i, _i, _i, _i, _f32p, _f32p, _i32p, _i32p, _f32p, _f32p],
    "orc_devox_grad": [_i, _i, _i, _i, _i32p, _f32p, _f32p, _f32p, _i],
    "orc_cube_vox": [_i, _i, _i, _i, _f32p, _i32p, _f32p, _i32p, _i32p],
    "orc_cube_devox": [_i, _i, _i, _i, _f32p, _f32p, _i32p, _f32p, _f32p],
    "orc_ball_query": [_i, _i, _i, _f, _i, _f32p, _f32p, _i32p],
    "orc_grouping": [_i, _i, _i, _i, _i, _f32p, _i32p, _f32p],
    "orc_grouping_grad": [_i, _i, _i, _i, _i, _f32p, _i32p, _f32p],
    "orc_local_ppf": [_i, _i, _i, _i, _f32p, _f32p, _f32p, _f32p, _i32p, _i, _i, _f32p],
    "orc_normalize_sph": [_i, _i, _f32p, _f32p],
    "orc_acosf_v": [_i, _f32p, _f32p],
    "orc_acosf_fast_v": [_i, _f32p, _f32p],
    "orc_atanf_v": [_i, _f32p, _f32p],
    "orc_acos_d_v": [_i, _f64p, _f64p],
    "orc_sph_index_v": [_i, _f32p, _i, _i, _i32p],
    "orc_sph_index_ulp": [_i, _f32p, _i, _i, _i, _i32p],
    "orc_mutual_nn": [_i, _i, _i, _i, _f32p, _f32p, _i32p, _i32p, _i32p, _i32p, _i32p],
    "orc_lrf": [_i, _i, _f32p, _f32p, _f32p, _i32p, _i32p],
    "orc_gather": [_i, _i, _i, _i, _f32p, _i32p, _f32p],
    "orc_gather_grad": [_i, _i, _i, _i, _f32p, _i32p, _f32p],
    "orc_fps": [_i, _i, _i, _f32p, _i32p],
    "orc_three_nn": [_i, _i, _i, _i, _f32p, _f32p, _f32p, _f32p, _i32p, _f32p],
    "orc_three_nn_grad": [_i, _i, _i, _i, _f32p, _i32p, _f32p, _f32p],
    "orc_normals": [_i, _i, ctypes.c_double, _f32p, _f32p, _i32p],
    "orc_num_threads": [],
    "orc_set_num_threads": [_i],
}


def build():
    """Compile the oracle with its Makefile (gcc; no GPU needed)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = _i if name == "orc_num_threads" else None
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def set_num_threads(t):
    lib().orc_set_num_threads(int(t))


def num_threads():
    return lib().orc_num_threads()


# ---------------------------------------------------------------- KNN
def knn_forward(xyz1, xyz2, k):
    """knn_forward_cuda (knn.cpp:6-25): both directions."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    d1 = np.empty((b, k, n), np.float32)
    i1 = np.empty((b, k, n), np.int32)
    d2 = np.empty((b, k, m), np.float32)
    i2 = np.empty((b, k, m), np.int32)
    lib().orc_knn_dir(b, c, n, m, k, xyz1, xyz2, d1, i1)
    lib().orc_knn_dir(b, c, m, n, k, xyz2, xyz1, d2, i2)
    return d1, d2, i1, i2


def knn_dir(xyz1, xyz2, k):
    """One direction of KnnKernel (knn.cu:5-49)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    d = np.empty((b, k, n), np.float32)
    i = np.empty((b, k, n), np.int32)
    lib().orc_knn_dir(b, c, n, m, k, xyz1, xyz2, d, i)
    return d, i


def knn_backward(xyz1, xyz2, gd1, gd2, idx1, idx2):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    k = idx1.shape[1]
    g1 = np.empty((b, c, n), np.float32)
    g2 = np.empty((b, c, m), np.float32)
    lib().orc_knn_grad(b, c, n, m, k, xyz1, xyz2, _f32(gd1), _f32(gd2), _i32(idx1), _i32(idx2), g1, g2)
    return g1, g2


# ---------------------------------------------------------------- PPF
def spherical_ppf_forward(coords, center, normals, center_normal):
    """spherical_ppf_forward (ppf.cpp:17-36): argument order of the backend."""
    coords = _f32(coords)
    b, _, n = coords.shape
    out = np.empty((b, 4, n), np.float32)
    lib().orc_global_ppf(b, n, coords, _f32(center), _f32(normals), _f32(center_normal), out)
    return out


def local_ppf(points, normals, centers, center_normals, idx, kmajor, relative=True):
    points = _f32(points)
    b, _, n = points.shape
    m = centers.shape[2]
    u = idx.shape[1] if kmajor else idx.shape[2]
    out = np.empty((b, 4, u, m), np.float32)
    lib().orc_local_ppf(b, n, m, u, points, _f32(normals), _f32(centers), _f32(center_normals),
                        _i32(idx), int(bool(kmajor)), int(bool(relative)), out)
    return out


# ------------------------------------------------------- voxelization
def spherical_avg_voxelize_forward(features, coords, r, use_fma=True):
    features, coords = _f32(features), _f32(coords)
    b, c, n = features.shape
    r3 = r ** 3
    out = np.empty((b, c, r3), np.float32)
    ind = np.empty((b, n), np.int32)
    cnt = np.empty((b, r3), np.int32)
    lib().orc_sph_vox(b, c, n, r, features, coords, out, ind, cnt, int(bool(use_fma)))
    return out, ind, cnt


def avg_voxelize_backward(grad_y, ind, cnt):
    grad_y = _f32(grad_y)
    b, c, r3 = grad_y.shape
    n = ind.shape[1]
    gx = np.empty((b, c, n), np.float32)
    lib().orc_avg_vox_grad(b, c, n, r3, _i32(ind), _i32(cnt), grad_y, gx)
    return gx


def spherical_trilinear_devoxelize_forward(r, coords, features, g_inds):
    coords, features = _f32(coords), _f32(features)
    b, c = features.shape[:2]
    n = coords.shape[2]
    inds = np.empty((b, 8, n), np.int32)
    wgts = np.empty((b, 8, n), np.float32)
    outs = np.empty((b, c, n), np.float32)
    lib().orc_sph_devox(b, c, n, r, coords, features.reshape(b, c, -1), _i32(g_inds), inds, wgts, outs)
    return outs, inds, wgts


def devoxelize_backward(grad_y, inds, wgts, r, spherical=True):
    grad_y = _f32(grad_y)
    b, c, n = grad_y.shape
    gx = np.empty((b, c, r ** 3), np.float32)
    lib().orc_devox_grad(b, c, n, r ** 3, _i32(inds), _f32(wgts), grad_y, gx, int(bool(spherical)))
    return gx


def avg_voxelize_forward(features, coords, r):
    features = _f32(features)
    b, c, n = features.shape
    r3 = r ** 3
    out = np.empty((b, c, r3), np.float32)
    ind = np.empty((b, n), np.int32)
    cnt = np.empty((b, r3), np.int32)
    lib().orc_cube_vox(b, c, n, r, features, _i32(coords), out, ind, cnt)
    return out, ind, cnt


def trilinear_devoxelize_forward(r, coords, features):
    coords, features = _f32(coords), _f32(features)
    b, c = features.shape[:2]
    n = coords.shape[2]
    inds = np.empty((b, 8, n), np.int32)
    wgts = np.empty((b, 8, n), np.float32)
    outs = np.empty((b, c, n), np.float32)
    lib().orc_cube_devox(b, c, n, r, coords, features.reshape(b, c, -1), inds, wgts, outs)
    return outs, inds, wgts


# ------------------------------------------------ ball query / grouping
def ball_query(centers, points, radius, u):
    centers, points = _f32(centers), _f32(points)
    b, _, m = centers.shape
    n = points.shape[2]
    idx = np.empty((b, m, u), np.int32)
    lib().orc_ball_query(b, n, m, float(radius), u, centers, points, idx)
    return idx


def grouping_forward(features, idx):
    features = _f32(features)
    b, c, n = features.shape
    _, m, u = idx.shape
    out = np.empty((b, c, m, u), np.float32)
    lib().orc_grouping(b, c, n, m, u, features, _i32(idx), out)
    return out


def grouping_backward(grad_y, idx, n):
    grad_y = _f32(grad_y)
    b, c, m, u = grad_y.shape
    gx = np.empty((b, c, n), np.float32)
    lib().orc_grouping_grad(b, c, n, m, u, grad_y, _i32(idx), gx)
    return gx


# ------------------------------------------------------- misc / math
def normalize_sph(coords):
    coords = _f32(coords)
    b, _, n = coords.shape
    out = np.empty_like(coords)
    lib().orc_normalize_sph(b, n, coords, out)
    return out


def acosf(x):
    x = _f32(x).ravel()
    y = np.empty_like(x)
    lib().orc_acosf_v(x.size, x, y)
    return y


def acosf_fast(x):
    """The local PPF's faithful fp32 acos (pcr_math.h pcr_acosf_fast)."""
    x = _f32(x).ravel()
    y = np.empty_like(x)
    lib().orc_acosf_fast_v(x.size, x, y)
    return y


def atanf(x):
    x = _f32(x).ravel()
    y = np.empty_like(x)
    lib().orc_atanf_v(x.size, x, y)
    return y


def acos_d(x):
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    y = np.empty_like(x)
    lib().orc_acos_d_v(x.size, x, y)
    return y


def sph_index(xyz, r, use_fma=True):
    """xyz: [3, n] normalised coords -> voxel index per point (-1 dropped)."""
    xyz = _f32(xyz)
    n = xyz.shape[1]
    ind = np.empty(n, np.int32)
    lib().orc_sph_index_v(n, xyz, r, int(bool(use_fma)), ind)
    return ind


def sph_index_ulp(xyz, r, dacos, datan):
    """sph_index with the float acos / atan results moved dacos / datan fp32
    ulps from the correctly rounded values (CUDA's float acosf / atanf are
    accurate to <= 2 ulp; spherical_vox.cu:46,54)."""
    xyz = _f32(xyz)
    n = xyz.shape[1]
    ind = np.empty(n, np.int32)
    lib().orc_sph_index_ulp(n, xyz, r, int(dacos), int(datan), ind)
    return ind


def mutual_nn(f1, f2):
    """Feature-space mutual nearest neighbours (datasets/deepgmr_mn40.py:
    232-244) of p pairs: f1 [p, n1, c], f2 [p, n2, c] -> corr12 [p, n1],
    corr21 [p, n2], idx1 [p, n1], idx2 [p, n1] (mutual pairs first, -1
    after), count [p]."""
    f1, f2 = _f32(f1), _f32(f2)
    p, n1, c = f1.shape
    n2 = f2.shape[1]
    corr12 = np.empty((p, n1), np.int32)
    corr21 = np.empty((p, n2), np.int32)
    idx1 = np.empty((p, n1), np.int32)
    idx2 = np.empty((p, n1), np.int32)
    count = np.empty((p,), np.int32)
    lib().orc_mutual_nn(p, n1, n2, c, f1, f2, corr12, corr21, idx1, idx2, count)
    return corr12, corr21, idx1, idx2, count


# ------------------------------------------------ LRF change_coords (f2)
def lrf_change_coords(coords):
    """models/pvcnn_classify.py:153-184: coords [b, 3, n] -> (new_coords
    [b, 3, n], basis [b, 3, 3] rows x/y/z, picks [b, 2], status [b])."""
    coords = _f32(coords)
    b, _, n = coords.shape
    out = np.empty_like(coords)
    basis = np.empty((b, 3, 3), np.float32)
    picks = np.empty((b, 2), np.int32)
    status = np.empty((b,), np.int32)
    lib().orc_lrf(b, n, coords, out, basis, picks, status)
    return out, basis, picks, status


# ------------------------------------------------ PointNet++ ops (f4)
def gather_features_forward(features, indices):
    """sampling.cpp gather_features_forward: [b, c, n] x [b, m] -> [b, c, m]."""
    features, indices = _f32(features), _i32(indices)
    b, c, n = features.shape
    m = indices.shape[1]
    out = np.empty((b, c, m), np.float32)
    lib().orc_gather(b, c, n, m, features, indices, out)
    return out


def gather_features_backward(grad_y, indices, n):
    grad_y, indices = _f32(grad_y), _i32(indices)
    b, c, m = grad_y.shape
    gx = np.empty((b, c, n), np.float32)
    lib().orc_gather_grad(b, c, n, m, grad_y, indices, gx)
    return gx


def furthest_point_sampling(coords, m):
    coords = _f32(coords)
    b, _, n = coords.shape
    idx = np.zeros((b, m), np.int32)
    lib().orc_fps(b, n, m, coords, idx)
    return idx


def three_nearest_neighbors_interpolate_forward(points, centers, centers_features):
    """neighbor_interpolate.cpp: -> (out [b, c, n], indices [b, 3, n],
    weights [b, 3, n])."""
    points, centers, cf = _f32(points), _f32(centers), _f32(centers_features)
    b, c, m = cf.shape
    n = points.shape[2]
    out = np.empty((b, c, n), np.float32)
    inds = np.empty((b, 3, n), np.int32)
    wgts = np.empty((b, 3, n), np.float32)
    lib().orc_three_nn(b, c, m, n, points, centers, cf, out, inds, wgts)
    return out, inds, wgts


def three_nearest_neighbors_interpolate_backward(grad_y, indices, weights, m):
    grad_y, indices, weights = _f32(grad_y), _i32(indices), _f32(weights)
    b, c, n = grad_y.shape
    gx = np.empty((b, c, m), np.float32)
    lib().orc_three_nn_grad(b, c, n, m, grad_y, indices, weights, gx)
    return gx


# ------------------------------------------- normal estimation (f3)
def estimate_normals(points, radius=0.1):
    """utils/open3d_func.py:77-83 restated: points [b, 3, n] -> (normals
    [b, 3, n], counts [b, n])."""
    points = _f32(points)
    b, _, n = points.shape
    normals = np.empty_like(points)
    counts = np.empty((b, n), np.int32)
    lib().orc_normals(b, n, float(radius), points, normals, counts)
    return normals, counts
