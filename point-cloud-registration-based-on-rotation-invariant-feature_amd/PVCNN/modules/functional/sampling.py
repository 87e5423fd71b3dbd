"""gather / furthest_point_sample / logits_mask (reference:
PVCNN/modules/functional/sampling.py:10-81) on the MI355X library."""
import numpy as np
import torch
from torch.autograd import Function

from .backend import _backend

__all__ = ["gather", "furthest_point_sample", "logits_mask"]


class Gather(Function):
    """features [B,C,N], indices [B,M] -> [B,C,M] (sampling.py:10-34)."""

    @staticmethod
    def forward(ctx, features, indices):
        features = features.contiguous()
        indices = indices.int().contiguous()
        ctx.save_for_backward(indices)
        ctx.num_points = features.size(-1)
        return _backend.gather_features_forward(features, indices)

    @staticmethod
    def backward(ctx, grad_output):
        (indices,) = ctx.saved_tensors
        grad = _backend.gather_features_backward(grad_output.contiguous(), indices, ctx.num_points)
        return grad, None


gather = Gather.apply


def furthest_point_sample(coords, num_samples):
    """coords [B,3,N] -> the coordinates of num_samples FPS centres [B,3,M]
    (sampling.py:37-47)."""
    coords = coords.contiguous()
    indices = _backend.furthest_point_sampling(coords, num_samples)
    return gather(coords, indices)


def logits_mask(coords, logits, num_points_per_object):
    """sampling.py:50-81: keep the points whose logit 1 beats logit 0, centre
    them, and draw num_points_per_object of them with numpy's global RNG (the
    reference's host-side sampling, kept as is: the draw is the caller's RNG
    stream, not device work).  Returns (selected [B,3,M], mean [B,3],
    mask [B,N])."""
    b, _, n = coords.shape
    mask = torch.lt(logits[:, 0, :], logits[:, 1, :])
    num_candidates = torch.sum(mask, dim=-1, keepdim=True)
    masked = coords * mask.view(b, 1, n)
    mean = torch.sum(masked, dim=-1) / torch.max(num_candidates,
                                                 torch.ones_like(num_candidates)).float()
    selected = torch.zeros((b, num_points_per_object), device=coords.device, dtype=torch.int32)
    for i in range(b):
        cand = mask[i].nonzero().view(-1)
        nc = cand.numel()
        if nc >= num_points_per_object:
            choice = np.random.choice(nc, num_points_per_object, replace=False)
            selected[i] = cand[torch.from_numpy(choice).to(cand.device)]
        elif nc > 0:
            choice = np.concatenate([
                np.arange(nc).repeat(num_points_per_object // nc),
                np.random.choice(nc, num_points_per_object % nc, replace=False)])
            np.random.shuffle(choice)
            selected[i] = cand[torch.from_numpy(choice).to(cand.device)]
    return gather(masked - mean.view(b, -1, 1), selected), mean, mask
