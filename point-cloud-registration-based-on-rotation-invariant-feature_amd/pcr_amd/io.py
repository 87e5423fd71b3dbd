"""Input side of the path: the reference's on-disk point
format, the ModelNet40 sample pipeline around it, and GPU normals.

- ``read_xyzn_txt`` is the native parser of libpcr_amd.so for the
  ``modelnet40_normal_resampled/*.txt`` rows (datasets/modelnet40.py:30).
- ``ModelNet40Dataset`` mirrors ``_ModelNet40Dataset`` (datasets/modelnet40.py:
  11-95): the class list, the split files, random point choice, centring and
  the optional random rotation, returning ``(pcd [3|6, n], target)``.
- ``random_rotation`` keeps the reference's quirk (utils/open3d_func.py:85-87):
  it reseeds numpy with ``seed=0`` on every call, so every sample gets the
  same rotation.
- ``get_normals`` is utils/open3d_func.py:77-83 on the GPU
  (``ops.estimate_normals``, radius 0.1).

The DeepGMR h5 test files (datasets/deepgmr_mn40.py:46-49) need h5py, which
is not installed; they are out of reach here.
"""
import ctypes
import os

import numpy as np

from . import _lib


def read_xyzn_txt(path):
    """np.loadtxt(path, delimiter=',').astype(np.float32), natively: ->
    float32 array [rows, cols]."""
    lib = _lib.load()
    p = os.fsencode(path)
    rows, cols = ctypes.c_longlong(0), ctypes.c_int(0)
    _lib.check(lib.pcr_txt_shape(p, ctypes.byref(rows), ctypes.byref(cols)), "txt_shape")
    out = np.empty((rows.value, max(cols.value, 1)), np.float32)
    if rows.value:
        _lib.check(lib.pcr_read_xyzn_txt(p, out.ctypes.data, rows.value, cols.value),
                   "read_xyzn_txt")
    return out


def randchoice(n, m):
    """utils/random_choice.py:2-7."""
    return np.random.choice(n, m, replace=n < m)


def random_rotation(points, normals=None, max_degree=360, max_amp=3, seed=0):
    """utils/open3d_func.py:85-104: a rotation about a random axis plus a
    random translation, drawn after np.random.seed(seed)."""
    from scipy.spatial.transform import Rotation
    np.random.seed(seed)
    x = np.random.rand(6)
    degree = np.random.rand(1) * max_degree * np.pi / 180
    amp = np.random.rand(1) * max_amp
    w, v = x[:3] / np.linalg.norm(x[:3]), x[3:] / np.linalg.norm(x[3:])
    w = w * degree
    v = v * amp
    r = Rotation.from_rotvec(w)
    pts = r.apply(points) + v[np.newaxis, :]
    t = np.eye(4)
    t[:3, :3] = r.as_matrix()
    t[:3, 3] = v
    if normals is not None:
        return t, pts.astype(np.float32), r.apply(normals).astype(np.float32)
    return t, pts.astype(np.float32)


class ModelNet40Dataset:
    """datasets/modelnet40.py:11-95 without the 'fps' cache files (the
    reference's host FPS helper does not run: utils/random_choice.py:22 calls
    np.randint).  Returns (pcd [6 or 3, num_points] float32, target int)."""

    def __init__(self, datadir, partition, shapenum, num_points, normalize=True,
                 with_normals=True, random_rot=False):
        self.rootdir = datadir
        self.num_points = num_points
        self.normalize = normalize
        self.with_normals = with_normals
        self.random_rot = random_rot
        with open(os.path.join(datadir, "modelnet%s_shape_names.txt" % shapenum)) as f:
            classes = sorted(line.strip() for line in f)
        self.classes = classes
        class_to_idx = {c: i for i, c in enumerate(classes)}
        self.samples = []
        with open(os.path.join(datadir, "modelnet%s_%s.txt" % (shapenum, partition))) as f:
            for line in f:
                name = line.strip()
                cls = name[:-5]
                self.samples.append((os.path.join(cls, name), class_to_idx[cls]))

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        sample, target = self.samples[index]
        pc = read_xyzn_txt(os.path.join(self.rootdir, sample + ".txt"))
        idx = randchoice(pc.shape[0], self.num_points)
        points = pc[idx, :3].copy()
        normals = pc[idx, 3:].copy()
        if self.normalize:
            points -= np.mean(points, axis=0, keepdims=True)
        if self.random_rot:
            if self.with_normals:
                _, points, normals = random_rotation(points, normals)
                pcd = np.concatenate((points, normals), axis=1)
            else:
                _, pcd = random_rotation(points)
        else:
            pcd = np.concatenate((points, normals), axis=1) if self.with_normals else points
        return pcd.T, target


def get_normals(points, radius=0.1):
    """utils/open3d_func.py:77-83 on the GPU.  points: [n, 3] (numpy or
    tensor, one cloud, as the reference) or a [b, 3, n] CUDA tensor ->
    normals of the same layout; numpy input gives a float32 numpy result."""
    import torch
    from . import ops
    if isinstance(points, np.ndarray):
        dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.from_numpy(np.ascontiguousarray(points.T, np.float32))[None].to(dev)
        return ops.estimate_normals(t, radius)[0].T.cpu().numpy()
    if points.dim() == 2:
        return ops.estimate_normals(points.t().contiguous()[None], radius)[0].t()
    return ops.estimate_normals(points.contiguous(), radius)
