"""Torch-tensor entry points of the MI355X hot path.

Each function reproduces one function of the reference's pybind11 module
``_multi_shape_pvcnn_backend`` (PVCNN/modules/functional/src/bindings.cpp:13-56)
-- same name, argument order, checks and return structure -- and calls the
C ABI of libpcr_amd.so on torch's current HIP stream.  Outputs are allocated
with ``torch.empty`` (the library writes every element, including the slots
the reference leaves at its ``torch::zeros`` / ``ones*10000`` fill).

Checks follow src/utils.hpp:15-28 (CHECK_CUDA / CHECK_CONTIGUOUS /
CHECK_IS_FLOAT / CHECK_IS_INT -> RuntimeError with the same messages).
"""
import torch

from . import _lib


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _check_cuda(t, name):
    if not t.is_cuda:
        raise RuntimeError("%s must be a CUDA tensor" % name)


def _check_contig(t, name):
    if not t.is_contiguous():
        raise RuntimeError("%s must be a contiguous tensor" % name)


def _check_float(t, name):
    if t.dtype != torch.float32:
        raise RuntimeError("%s must be a float tensor" % name)


def _check_int(t, name):
    if t.dtype != torch.int32:
        raise RuntimeError("%s must be an int tensor" % name)


def _check(t, name, kind="float"):
    _check_cuda(t, name)
    _check_contig(t, name)
    if kind == "float":
        _check_float(t, name)
    elif kind == "int":
        _check_int(t, name)


def _workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------ KNN
def knn_forward_cuda(xyz1, xyz2, k):
    """knn/knn.cpp:6-25 -> [dist1, dist2, idx1, idx2]."""
    _check(xyz1, "xyz1")
    _check(xyz2, "xyz2")
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    k = int(k)
    dev = xyz1.device
    dist1 = torch.empty((b, k, n), dtype=torch.float32, device=dev)
    dist2 = torch.empty((b, k, m), dtype=torch.float32, device=dev)
    idx1 = torch.empty((b, k, n), dtype=torch.int32, device=dev)
    idx2 = torch.empty((b, k, m), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _workspace(lib.pcr_knn_workspace_size(b, n, m), dev)
    _lib.check(lib.pcr_knn_forward(
        _ptr(xyz1), _ptr(xyz2), b, c, n, m, k, _ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2),
        _ptr(ws), ws.numel(), _stream()), "knn_forward_cuda")
    return [dist1, dist2, idx1, idx2]


def knn_backward_cuda(xyz1, xyz2, graddist1, graddist2, idx1, idx2):
    """knn/knn.cpp:27-52 -> [gradxyz1, gradxyz2]."""
    _check(xyz1, "xyz1")
    _check(xyz2, "xyz2")
    _check(graddist1, "graddist1")
    _check(graddist2, "graddist2")
    _check(idx1, "idx1", "int")
    _check(idx2, "idx2", "int")
    b, c, n = xyz1.shape
    m = xyz2.shape[2]
    k = idx1.shape[1]
    g1 = torch.empty((b, c, n), dtype=torch.float32, device=xyz1.device)
    g2 = torch.empty((b, c, m), dtype=torch.float32, device=xyz1.device)
    # the atomics-free path: (query, slot) pairs counting-sorted by neighbour
    # in a workspace, then one gather per point (bit-repeatable)
    lib = _lib.load()
    ws = torch.empty(lib.pcr_knn_backward_workspace_size(b, n, m, k), dtype=torch.uint8,
                     device=xyz1.device)
    _lib.check(lib.pcr_knn_backward_ws(
        _ptr(xyz1), _ptr(xyz2), _ptr(graddist1), _ptr(graddist2), _ptr(idx1), _ptr(idx2),
        b, c, n, m, k, _ptr(g1), _ptr(g2), _ptr(ws), ws.numel(), _stream()),
        "knn_backward_cuda")
    return [g1, g2]


# ------------------------------------------------------------------ PPF
def spherical_ppf_forward(coords, center, normals, center_normal):
    """spherical_ppf/ppf.cpp:17-36 -> feat [b, 4, n]."""
    for t, nm in ((coords, "coords"), (center, "center"), (normals, "normals"),
                  (center_normal, "center_normal")):
        _check(t, nm)
    b, _, n = coords.shape
    feat = torch.empty((b, 4, n), dtype=torch.float32, device=coords.device)
    _lib.check(_lib.load().pcr_spherical_ppf_forward(
        _ptr(coords), _ptr(center), _ptr(normals), _ptr(center_normal), b, n, _ptr(feat),
        _stream()), "spherical_ppf_forward")
    return feat


def local_ppf_forward(points, normals, centers, center_normals, indices, kmajor=False,
                      relative=True):
    """Fused grouping + local PPF of pvcnn_classify.py:252-269 -> [b, 4, u, m]."""
    for t, nm in ((points, "points"), (normals, "normals"), (centers, "centers"),
                  (center_normals, "center_normals")):
        _check(t, nm)
    _check(indices, "indices", "int")
    b, _, n = points.shape
    m = centers.shape[2]
    u = indices.shape[1] if kmajor else indices.shape[2]
    out = torch.empty((b, 4, u, m), dtype=torch.float32, device=points.device)
    _lib.check(_lib.load().pcr_local_ppf_forward(
        _ptr(points), _ptr(normals), _ptr(centers), _ptr(center_normals), _ptr(indices),
        b, n, m, u, int(bool(kmajor)), int(bool(relative)), _ptr(out), _stream()),
        "local_ppf_forward")
    return out


def knn_local_ppf(xyz, normals, k, relative=True, want_dist=False):
    """Fused self-KNN + local PPF -> (idx [b,k,n], ppf [b,4,k,n], dist or None)."""
    _check(xyz, "xyz")
    _check(normals, "normals")
    b, _, n = xyz.shape
    dev = xyz.device
    idx = torch.empty((b, k, n), dtype=torch.int32, device=dev)
    ppf = torch.empty((b, 4, k, n), dtype=torch.float32, device=dev)
    dist = torch.empty((b, k, n), dtype=torch.float32, device=dev) if want_dist else None
    lib = _lib.load()
    ws = _workspace(lib.pcr_knn_workspace_size(b, n, n), dev)
    _lib.check(lib.pcr_knn_local_ppf(
        _ptr(xyz), _ptr(normals), b, n, int(k), int(bool(relative)), _ptr(idx), _ptr(dist),
        _ptr(ppf), _ptr(ws), ws.numel(), _stream()), "knn_local_ppf")
    return idx, ppf, dist


# -------------------------------------------------- ball query / grouping
def ball_query(centers_coords, points_coords, radius, num_neighbors):
    """ball_query/ball_query.cpp:6-30 -> idx [b, m, u]."""
    _check(centers_coords, "centers_coords")
    _check(points_coords, "points_coords")
    b, _, m = centers_coords.shape
    n = points_coords.shape[2]
    u = int(num_neighbors)
    idx = torch.empty((b, m, u), dtype=torch.int32, device=centers_coords.device)
    _lib.check(_lib.load().pcr_ball_query(
        _ptr(centers_coords), _ptr(points_coords), b, m, n, float(radius), u, _ptr(idx),
        _stream()), "ball_query")
    return idx


def grouping_forward(features, indices):
    """grouping/grouping.cpp:6-24 -> [b, c, m, u]."""
    _check(features, "features")
    _check(indices, "indices", "int")
    b, c, n = features.shape
    m, u = indices.shape[1], indices.shape[2]
    out = torch.empty((b, c, m, u), dtype=torch.float32, device=features.device)
    _lib.check(_lib.load().pcr_grouping_forward(
        _ptr(features), _ptr(indices), b, c, n, m, u, _ptr(out), _stream()), "grouping_forward")
    return out


def grouping_backward(grad_y, indices, n):
    """grouping/grouping.cpp:26-44 -> [b, c, n]."""
    _check(grad_y, "grad_y")
    _check(indices, "indices", "int")
    b, c = grad_y.shape[:2]
    m, u = indices.shape[1], indices.shape[2]
    gx = torch.empty((b, c, int(n)), dtype=torch.float32, device=grad_y.device)
    _lib.check(_lib.load().pcr_grouping_backward(
        _ptr(grad_y), _ptr(indices), b, c, int(n), m, u, _ptr(gx), _stream()),
        "grouping_backward")
    return gx


# ----------------------------------------------------------- voxelization
def spherical_avg_voxelize_forward(features, coords, resolution):
    """spherical_voxelization/spherical_vox.cpp:17-46 -> [out, ind, cnt]."""
    _check(features, "features")
    _check(coords, "coords")
    b, c, n = features.shape
    r = int(resolution)
    r3 = r * r * r
    dev = features.device
    out = torch.empty((b, c, r3), dtype=torch.float32, device=dev)
    ind = torch.empty((b, n), dtype=torch.int32, device=dev)
    cnt = torch.empty((b, r3), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _workspace(lib.pcr_voxelize_workspace_size_c(b, c, n, r), dev)
    _lib.check(lib.pcr_spherical_avg_voxelize_forward(
        _ptr(features), _ptr(coords), b, c, n, r, _ptr(out), _ptr(ind), _ptr(cnt), _ptr(ws),
        ws.numel(), _stream()), "spherical_avg_voxelize_forward")
    return [out, ind, cnt]


def avg_voxelize_forward(features, coords, resolution):
    """voxelization/vox.cpp:17-46 (int voxel coords) -> [out, ind, cnt]."""
    _check(features, "features")
    _check(coords, "coords", "int")
    b, c, n = features.shape
    r = int(resolution)
    r3 = r * r * r
    dev = features.device
    out = torch.empty((b, c, r3), dtype=torch.float32, device=dev)
    ind = torch.empty((b, n), dtype=torch.int32, device=dev)
    cnt = torch.empty((b, r3), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _workspace(lib.pcr_voxelize_workspace_size_c(b, c, n, r), dev)
    _lib.check(lib.pcr_avg_voxelize_forward(
        _ptr(features), _ptr(coords), b, c, n, r, _ptr(out), _ptr(ind), _ptr(cnt), _ptr(ws),
        ws.numel(), _stream()), "avg_voxelize_forward")
    return [out, ind, cnt]


def _avg_vox_backward(grad_y, indices, cnt, what):
    _check(grad_y, "grad_y")
    _check(indices, "indices", "int")
    _check(cnt, "cnt", "int")
    b, c, s = grad_y.shape
    n = indices.shape[1]
    gx = torch.empty((b, c, n), dtype=torch.float32, device=grad_y.device)
    _lib.check(_lib.load().pcr_avg_voxelize_backward(
        _ptr(grad_y), _ptr(indices), _ptr(cnt), b, c, n, s, _ptr(gx), _stream()), what)
    return gx


def spherical_avg_voxelize_backward(grad_y, indices, cnt):
    """spherical_vox.cpp:57-79 -> grad_x [b, c, n]."""
    return _avg_vox_backward(grad_y, indices, cnt, "spherical_avg_voxelize_backward")


def avg_voxelize_backward(grad_y, indices, cnt):
    """vox.cpp:57-76 -> grad_x [b, c, n]."""
    return _avg_vox_backward(grad_y, indices, cnt, "avg_voxelize_backward")


def spherical_normalize(coords):
    """Spherical_Voxelization's normalisation (modules/spherical_vox.py:16-20)."""
    _check(coords, "coords")
    b, _, n = coords.shape
    out = torch.empty_like(coords)
    _lib.check(_lib.load().pcr_spherical_normalize(_ptr(coords), b, n, _ptr(out), _stream()),
               "spherical_normalize")
    return out


# --------------------------------------------------------- devoxelization
def spherical_trilinear_devoxelize_forward(r, is_training, coords, features, g_inds):
    """interpolate/spherical_trilinear_devox.cpp:19-56 -> [outs, inds, wgts]."""
    _check(features, "features")
    _check(coords, "coords")
    _check_cuda(g_inds, "g_inds")
    g_inds = g_inds.contiguous()
    if g_inds.dtype != torch.int32:
        raise RuntimeError("g_inds must be an int tensor")
    b, c = features.shape[:2]
    n = coords.shape[2]
    dev = features.device
    outs = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    inds = torch.empty((b, 8, n), dtype=torch.int32, device=dev)
    wgts = torch.empty((b, 8, n), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().pcr_spherical_trilinear_devoxelize_forward(
        int(r), int(bool(is_training)), _ptr(coords), _ptr(features), _ptr(g_inds), b, c, n,
        _ptr(outs), _ptr(inds), _ptr(wgts), _stream()), "spherical_trilinear_devoxelize_forward")
    return [outs, inds, wgts]


def trilinear_devoxelize_forward(r, is_training, coords, features):
    """interpolate/trilinear_devox.cpp:18-56 -> [outs, inds, wgts]."""
    _check(features, "features")
    _check(coords, "coords")
    b, c = features.shape[:2]
    n = coords.shape[2]
    dev = features.device
    outs = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    inds = torch.empty((b, 8, n), dtype=torch.int32, device=dev)
    wgts = torch.empty((b, 8, n), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().pcr_trilinear_devoxelize_forward(
        int(r), int(bool(is_training)), _ptr(coords), _ptr(features), b, c, n, _ptr(outs),
        _ptr(inds), _ptr(wgts), _stream()), "trilinear_devoxelize_forward")
    return [outs, inds, wgts]


def _devox_backward(grad_y, indices, weights, r, spherical, what):
    _check(grad_y, "grad_y")
    _check(weights, "weights")
    _check(indices, "indices", "int")
    b, c, n = grad_y.shape
    r = int(r)
    gx = torch.empty((b, c, r * r * r), dtype=torch.float32, device=grad_y.device)
    lib = _lib.load()
    ws = _workspace(lib.pcr_devoxelize_backward_workspace_size_r(b, n, r, int(spherical)),
                    grad_y.device)
    _lib.check(lib.pcr_devoxelize_backward_ws(
        _ptr(grad_y), _ptr(indices), _ptr(weights), b, c, n, r, int(spherical), _ptr(gx),
        _ptr(ws), ws.numel(), _stream()), what)
    return gx


def spherical_trilinear_devoxelize_backward(grad_y, indices, weights, r):
    """spherical_trilinear_devox.cpp:68-92 -> grad_x [b, c, r^3]."""
    return _devox_backward(grad_y, indices, weights, r, True,
                           "spherical_trilinear_devoxelize_backward")


def trilinear_devoxelize_backward(grad_y, indices, weights, r):
    """trilinear_devox.cpp:58-91 -> grad_x [b, c, r^3]."""
    return _devox_backward(grad_y, indices, weights, r, False, "trilinear_devoxelize_backward")


def dgcnn_center_gather(features, avg_grid, ind):
    """PVConv dgcnn centre term (modules/pvconv.py:68-89) -> related [b, c, n]."""
    _check(features, "features")
    _check(avg_grid, "avg_grid")
    _check(ind, "ind", "int")
    b, c, n = features.shape
    r3 = avg_grid.shape[2]
    out = torch.empty_like(features)
    _lib.check(_lib.load().pcr_dgcnn_center_gather(
        _ptr(features), _ptr(avg_grid), _ptr(ind), b, c, n, r3, _ptr(out), _stream()),
        "dgcnn_center_gather")
    return out


# ---------------------------------------------- PointNet++ ops (8f f4)
def gather_features_forward(features, indices):
    """sampling/sampling.cpp:6-23 -> out [b, c, m]."""
    _check(features, "features")
    _check(indices, "indices", "int")
    b, c, n = features.shape
    m = indices.shape[1]
    out = torch.empty((b, c, m), dtype=torch.float32, device=features.device)
    _lib.check(_lib.load().pcr_gather_features_forward(
        _ptr(features), _ptr(indices), b, c, n, m, _ptr(out), _stream()),
        "gather_features_forward")
    return out


def gather_features_backward(grad_y, indices, n):
    """sampling/sampling.cpp:25-41 -> grad_x [b, c, n]."""
    _check(grad_y, "grad_y")
    _check(indices, "indices", "int")
    b, c, m = grad_y.shape
    n = int(n)
    gx = torch.empty((b, c, n), dtype=torch.float32, device=grad_y.device)
    _lib.check(_lib.load().pcr_gather_features_backward(
        _ptr(grad_y), _ptr(indices), b, c, n, m, _ptr(gx), _stream()),
        "gather_features_backward")
    return gx


def furthest_point_sampling(coords, num_samples):
    """sampling/sampling.cpp:43-58 (bound as ``furthest_point_sampling``,
    bindings.cpp:18) -> indices [b, num_samples] int32."""
    _check(coords, "coords")
    b, _, n = coords.shape
    m = int(num_samples)
    dev = coords.device
    idx = torch.empty((b, m), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _workspace(lib.pcr_fps_workspace_size(b, n), dev)
    _lib.check(lib.pcr_furthest_point_sampling(
        _ptr(coords), b, n, m, _ptr(idx), _ptr(ws), ws.numel(), _stream()),
        "furthest_point_sampling")
    return idx


def three_nearest_neighbors_interpolate_forward(points_coords, centers_coords, centers_features):
    """interpolate/neighbor_interpolate.cpp:6-40 -> [out, indices, weights]."""
    _check(points_coords, "points_coords")
    _check(centers_coords, "centers_coords")
    _check(centers_features, "centers_features")
    b, c, m = centers_features.shape
    n = points_coords.shape[2]
    dev = points_coords.device
    out = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    inds = torch.empty((b, 3, n), dtype=torch.int32, device=dev)
    wgts = torch.empty((b, 3, n), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().pcr_three_nn_interpolate_forward(
        _ptr(points_coords), _ptr(centers_coords), _ptr(centers_features), b, c, m, n,
        _ptr(out), _ptr(inds), _ptr(wgts), _stream()),
        "three_nearest_neighbors_interpolate_forward")
    return [out, inds, wgts]


def three_nearest_neighbors_interpolate_backward(grad_y, indices, weights, m):
    """interpolate/neighbor_interpolate.cpp:42-65 -> grad_x [b, c, m]."""
    _check(grad_y, "grad_y")
    _check(indices, "indices", "int")
    _check(weights, "weights")
    b, c, n = grad_y.shape
    m = int(m)
    gx = torch.empty((b, c, m), dtype=torch.float32, device=grad_y.device)
    _lib.check(_lib.load().pcr_three_nn_interpolate_backward(
        _ptr(grad_y), _ptr(indices), _ptr(weights), b, c, n, m, _ptr(gx), _stream()),
        "three_nearest_neighbors_interpolate_backward")
    return gx


# ------------------------------------------ LRF change_coords (8f f2)
class LRFAssertionError(AssertionError):
    """One of the reference's change_coords asserts (pvcnn_classify.py:159,
    :169, :177) fired for some cloud."""


_LRF_MSG = {1: "base_x.norm() <= 1e-5 (pvcnn_classify.py:159)",
            2: "no base_y with |lambda| < 0.9 (pvcnn_classify.py:169)",
            3: "degenerate Gram-Schmidt, |base_x| < 1e-5 (pvcnn_classify.py:177)"}


def lrf_change_coords(coords, check=True, return_basis=False):
    """rot_invariant_preprocess == 'change_coords' (models/pvcnn_classify.py:
    153-184): coords [b, 3, n] -> new_coords [b, 3, n] in each cloud's local
    frame.  With ``check`` the per-cloud status is read back (one host sync,
    as the reference's asserts) and LRFAssertionError raised on a failure.
    ``return_basis`` also returns (basis [b, 3, 3], picks [b, 2], status [b])."""
    _check(coords, "coords")
    if coords.dim() != 3 or coords.shape[1] != 3:
        raise RuntimeError("lrf_change_coords: expected coords [b, 3, n]")
    b, _, n = coords.shape
    dev = coords.device
    out = torch.empty_like(coords)
    basis = torch.empty((b, 3, 3), dtype=torch.float32, device=dev)
    picks = torch.empty((b, 2), dtype=torch.int32, device=dev)
    status = torch.empty((b,), dtype=torch.int32, device=dev)
    _lib.check(_lib.load().pcr_lrf_change_coords(
        _ptr(coords), b, n, _ptr(out), _ptr(basis), _ptr(picks), _ptr(status), _stream()),
        "lrf_change_coords")
    if check and b > 0:
        st = status.cpu()
        bad = torch.nonzero(st).flatten().tolist()
        if bad:
            raise LRFAssertionError("change_coords: cloud %d: %s" % (bad[0], _LRF_MSG[int(st[bad[0]])]))
    if return_basis:
        return out, (basis, picks, status)
    return out


# ------------------------------------------ normal estimation (8f f3)
def estimate_normals(points, radius=0.1, return_counts=False):
    """get_normals (utils/open3d_func.py:77-83) for a batch on the GPU:
    points [b, 3, n] -> unit normals [b, 3, n] from the PCA of each point's
    radius neighbourhood, flipped to face the origin (Open3D's
    orient_normals_towards_camera_location default), (0, 0, 1) with fewer
    than 3 neighbours.  ``return_counts`` also returns the neighbour counts
    [b, n] int32."""
    _check(points, "points")
    if points.dim() != 3 or points.shape[1] != 3:
        raise RuntimeError("estimate_normals: expected points [b, 3, n]")
    b, _, n = points.shape
    normals = torch.empty_like(points)
    counts = torch.empty((b, n), dtype=torch.int32, device=points.device)
    _lib.check(_lib.load().pcr_estimate_normals(
        _ptr(points), b, n, float(radius), _ptr(normals), _ptr(counts), _stream()),
        "estimate_normals")
    return (normals, counts) if return_counts else normals


def mutual_nn_match(feat1, feat2, channel_major=False, workspace=None):
    """Feature-space mutual nearest neighbours of p registration pairs
    (datasets/deepgmr_mn40.py:232-244, batched): feat1 [p, n1, c],
    feat2 [p, n2, c] -> (corr12 [p, n1], corr21 [p, n2], idx1 [p, n1],
    idx2 [p, n1], count [p]); the first count[q] entries of idx1[q] / idx2[q]
    are the mutual pairs in ascending idx1, the rest -1.  channel_major:
    feat1 [p, c, n1], feat2 [p, c, n2] (the extractor's per-point layout),
    matched in place."""
    _check(feat1, "feat1")
    _check(feat2, "feat2")
    if feat1.dim() != 3 or feat2.dim() != 3 or feat1.shape[0] != feat2.shape[0]:
        raise RuntimeError("mutual_nn_match: expected 3-d features with equal pair counts")
    if channel_major:
        p, c, n1 = feat1.shape
        n2, c2 = feat2.shape[2], feat2.shape[1]
    else:
        p, n1, c = feat1.shape
        n2, c2 = feat2.shape[1], feat2.shape[2]
    if c != c2:
        raise RuntimeError("mutual_nn_match: channel counts differ (%d vs %d)" % (c, c2))
    dev = feat1.device
    i32 = dict(dtype=torch.int32, device=dev)
    corr12, corr21 = torch.empty((p, n1), **i32), torch.empty((p, n2), **i32)
    idx1, idx2 = torch.empty((p, n1), **i32), torch.empty((p, n1), **i32)
    count = torch.empty((p,), **i32)
    lib = _lib.load()
    need = max(256, lib.pcr_mutual_nn_workspace_size(p, n1, n2))
    ws = workspace if workspace is not None and workspace.numel() >= need else \
        torch.empty(need, dtype=torch.uint8, device=dev)
    fn = lib.pcr_mutual_nn_match_cm if channel_major else lib.pcr_mutual_nn_match
    _lib.check(fn(_ptr(feat1), _ptr(feat2), p, n1, n2, c, _ptr(corr12), _ptr(corr21),
                  _ptr(idx1), _ptr(idx2), _ptr(count), _ptr(ws), ws.numel(), _stream()),
               "mutual_nn_match")
    return corr12, corr21, idx1, idx2, count


def find_correspondence_one_pair(feat1, feat2):
    """datasets/deepgmr_mn40.py:232-244 on the GPU: feat1 [n1, c],
    feat2 [n2, c] -> (idx1, idx2), the mutual nearest neighbours in feature
    space (int64 tensors on the features' device, ascending idx1)."""
    _, _, idx1, idx2, count = mutual_nn_match(feat1.unsqueeze(0), feat2.unsqueeze(0))
    n = int(count[0].item())
    return idx1[0, :n].long(), idx2[0, :n].long()
