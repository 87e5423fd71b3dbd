"""spherical_avg_voxelize (reference: PVCNN/modules/functional/spherical_vox.py:8-40)."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["spherical_avg_voxelize", "Spherical_AvgVoxelization"]


class Spherical_AvgVoxelization(Function):
    """features [B,C,N], normalised coords [B,3,N] -> (grid [B,C,R,R,R],
    voxel index [B,N], -1 for dropped points)."""

    @staticmethod
    def forward(ctx, features, coords, resolution):
        features = features.contiguous()
        coords = coords.contiguous()
        b, c, n = features.shape
        out, indices, counts = _backend.spherical_avg_voxelize_forward(features, coords,
                                                                      resolution)
        ctx.mark_non_differentiable(indices)
        ctx.save_for_backward(indices, counts)
        r = resolution
        return out.view(b, c, r, r, r), indices.view(b, n)

    @staticmethod
    def backward(ctx, grad_output, _grad_ind):
        indices, counts = ctx.saved_tensors
        b, c = grad_output.shape[:2]
        grad = _backend.spherical_avg_voxelize_backward(
            grad_output.contiguous().view(b, c, -1), indices, counts)
        return grad, None, None


spherical_avg_voxelize = Spherical_AvgVoxelization.apply
