"""avg_voxelize (reference: PVCNN/modules/functional/voxelization.py:8-43), cube grid."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["avg_voxelize", "AvgVoxelization"]


class AvgVoxelization(Function):
    @staticmethod
    def forward(ctx, features, coords, resolution):
        features = features.contiguous()
        coords = coords.int().contiguous()
        b, c, n = features.shape
        out, indices, counts = _backend.avg_voxelize_forward(features, coords, resolution)
        ctx.mark_non_differentiable(indices)
        ctx.save_for_backward(indices, counts)
        r = resolution
        return out.view(b, c, r, r, r), indices.view(b, n)

    @staticmethod
    def backward(ctx, grad_output, _grad_ind):
        indices, counts = ctx.saved_tensors
        b, c = grad_output.shape[:2]
        grad = _backend.avg_voxelize_backward(grad_output.contiguous().view(b, c, -1), indices,
                                              counts)
        return grad, None, None


avg_voxelize = AvgVoxelization.apply
