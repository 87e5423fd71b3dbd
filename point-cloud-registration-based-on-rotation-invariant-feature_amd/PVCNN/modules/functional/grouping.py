"""grouping (reference: PVCNN/modules/functional/grouping.py:8-31)."""
from torch.autograd import Function

from .backend import _backend

__all__ = ["grouping", "Grouping"]


class Grouping(Function):
    """features [B,C,N], indices [B,M,U] -> [B,C,M,U]."""

    @staticmethod
    def forward(ctx, features, indices):
        features = features.contiguous()
        indices = indices.contiguous()
        ctx.save_for_backward(indices)
        ctx.num_points = features.size(-1)
        return _backend.grouping_forward(features, indices)

    @staticmethod
    def backward(ctx, grad_output):
        (indices,) = ctx.saved_tensors
        return _backend.grouping_backward(grad_output.contiguous(), indices, ctx.num_points), None


grouping = Grouping.apply
