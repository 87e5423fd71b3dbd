"""nearest_neighbor_interpolate (reference:
PVCNN/modules/functional/interpolatation.py:8-38; the file name keeps the
reference's spelling so its import path works unchanged)."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["nearest_neighbor_interpolate", "NeighborInterpolation"]


class NeighborInterpolation(Function):
    """points [B,3,N], centers [B,3,M], centers_features [B,C,M] -> [B,C,N]:
    inverse-squared-distance weights of the 3 nearest centres."""

    @staticmethod
    def forward(ctx, points_coords, centers_coords, centers_features):
        points_coords = points_coords.contiguous()
        centers_coords = centers_coords.contiguous()
        centers_features = centers_features.contiguous()
        out, indices, weights = _backend.three_nearest_neighbors_interpolate_forward(
            points_coords, centers_coords, centers_features)
        ctx.save_for_backward(indices, weights)
        ctx.num_centers = centers_coords.size(-1)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        indices, weights = ctx.saved_tensors
        grad = _backend.three_nearest_neighbors_interpolate_backward(
            grad_output.contiguous(), indices, weights, ctx.num_centers)
        return None, None, grad


nearest_neighbor_interpolate = NeighborInterpolation.apply
