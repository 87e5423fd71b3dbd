"""ppf (reference: PVCNN/modules/functional/ppf.py:8-22): global point-pair
feature of every point against its centre, [b, 4, n].  Not differentiable,
like the reference (a plain function, no autograd.Function)."""
from .backend import _backend

__all__ = ["ppf"]


def ppf(centers_coords, points_coords, centers_normals, points_normals):
    # the backend takes points first (spherical_ppf/ppf.cpp:17-20)
    return _backend.spherical_ppf_forward(points_coords.contiguous(), centers_coords.contiguous(),
                                          points_normals.contiguous(),
                                          centers_normals.contiguous())
