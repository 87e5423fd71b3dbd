"""trilinear_devoxelize (reference: PVCNN/modules/functional/devoxelization.py:8-44), cube grid."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["trilinear_devoxelize", "TrilinearDevoxelization"]


class TrilinearDevoxelization(Function):
    @staticmethod
    def forward(ctx, features, coords, resolution, is_training=True):
        b, c = features.shape[:2]
        features = features.contiguous().view(b, c, -1)
        coords = coords.contiguous()
        outs, inds, wgts = _backend.trilinear_devoxelize_forward(resolution, is_training, coords,
                                                                 features)
        ctx.save_for_backward(inds, wgts)
        ctx.r = resolution
        return outs

    @staticmethod
    def backward(ctx, grad_output):
        inds, wgts = ctx.saved_tensors
        r = ctx.r
        grad = _backend.trilinear_devoxelize_backward(grad_output.contiguous(), inds, wgts, r)
        return grad.view(grad_output.size(0), grad_output.size(1), r, r, r), None, None, None


trilinear_devoxelize = TrilinearDevoxelization.apply
