"""spherical_trilinear_devoxelize (reference:
PVCNN/modules/functional/spherical_devox.py:8-41)."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["spherical_trilinear_devoxelize", "Spherical_TrilinearDevoxelization"]


class Spherical_TrilinearDevoxelization(Function):
    """grid features [B,C,R,R,R] sampled at the points' spherical corners
    (reference quirks preserved, see include/pcr_math.h pcr_sph_corners)."""

    @staticmethod
    def forward(ctx, features, coords, g_inds, resolution, is_training=True):
        b, c = features.shape[:2]
        features = features.contiguous().view(b, c, -1)
        coords = coords.contiguous()
        outs, inds, wgts = _backend.spherical_trilinear_devoxelize_forward(
            resolution, is_training, coords, features, g_inds)
        ctx.save_for_backward(inds, wgts)
        ctx.r = resolution
        return outs

    @staticmethod
    def backward(ctx, grad_output):
        inds, wgts = ctx.saved_tensors
        r = ctx.r
        grad = _backend.spherical_trilinear_devoxelize_backward(grad_output.contiguous(), inds,
                                                                wgts, r)
        return grad.view(grad_output.size(0), grad_output.size(1), r, r, r), None, None, None, None


spherical_trilinear_devoxelize = Spherical_TrilinearDevoxelization.apply
