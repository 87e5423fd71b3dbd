"""``_backend`` of the reference (PVCNN/modules/functional/backend.py:14-39).

The reference JIT-compiles its CUDA sources into the pybind11 module
``_multi_shape_pvcnn_backend`` at import time.  Here ``_backend`` is the
prebuilt MI355X library (libpcr_amd.so, loaded eagerly so a missing build
fails at import exactly like a failed JIT build would), exposed with the same
function names and signatures (src/bindings.cpp:13-56).
"""
import types

from pcr_amd import _lib, ops

_lib.load()

_NAMES = [
    "gather_features_forward", "gather_features_backward", "furthest_point_sampling",
    "ball_query", "grouping_forward", "grouping_backward",
    "three_nearest_neighbors_interpolate_forward", "three_nearest_neighbors_interpolate_backward",
    "trilinear_devoxelize_forward", "trilinear_devoxelize_backward",
    "avg_voxelize_forward", "avg_voxelize_backward",
    "spherical_avg_voxelize_forward", "spherical_avg_voxelize_backward",
    "spherical_trilinear_devoxelize_forward", "spherical_trilinear_devoxelize_backward",
    "spherical_ppf_forward", "knn_forward_cuda", "knn_backward_cuda",
]

_backend = types.SimpleNamespace(**{name: getattr(ops, name) for name in _NAMES})

__all__ = ["_backend"]
