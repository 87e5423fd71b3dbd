"""ball_query (reference: PVCNN/modules/functional/ball_query.py:8-19)."""
from .backend import _backend

__all__ = ["ball_query"]


def ball_query(centers_coords, points_coords, radius, num_neighbors):
    """First `num_neighbors` points (index order) within `radius` of each
    centre, excluding d^2 <= 1e-5; unfilled slots repeat the first hit (0 if
    none).  -> IntTensor [B, M, U]."""
    return _backend.ball_query(centers_coords.contiguous(), points_coords.contiguous(), radius,
                               num_neighbors)
