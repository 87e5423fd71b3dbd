"""k_nearest_neighbor (reference: PVCNN/modules/functional/knn.py:6-26)."""
import torch

from .backend import _backend

__all__ = ["k_nearest_neighbor", "K_Nearest_Neighbor"]


class K_Nearest_Neighbor(torch.autograd.Function):
    """Both-direction KNN; returns squared distances and indices, k-major
    [b, k, n] / [b, k, m].  Indices are non-differentiable; the backward
    routes dist gradients to both point sets (knn.cu:52-78)."""

    @staticmethod
    def forward(ctx, xyz1, xyz2, k):
        xyz1 = xyz1.float().contiguous()
        xyz2 = xyz2.float().contiguous()
        dist1, dist2, idx1, idx2 = _backend.knn_forward_cuda(xyz1, xyz2, k)
        ctx.mark_non_differentiable(idx1, idx2)
        ctx.save_for_backward(xyz1, xyz2, idx1, idx2)
        return dist1, dist2, idx1, idx2

    @staticmethod
    def backward(ctx, graddist1, graddist2, _gi1, _gi2):
        xyz1, xyz2, idx1, idx2 = ctx.saved_tensors
        g1, g2 = _backend.knn_backward_cuda(xyz1, xyz2, graddist1.contiguous(),
                                            graddist2.contiguous(), idx1, idx2)
        return g1, g2, None


k_nearest_neighbor = K_Nearest_Neighbor.apply
