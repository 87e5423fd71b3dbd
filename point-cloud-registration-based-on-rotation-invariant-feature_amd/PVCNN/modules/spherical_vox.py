"""Spherical_Voxelization (reference: PVCNN/modules/spherical_vox.py:9-26)."""
import torch.nn as nn

from . import functional as F

__all__ = ["Spherical_Voxelization"]


class Spherical_Voxelization(nn.Module):
    """Centre the cloud, scale its farthest point to radius ~1, then
    spherical-average-voxelize.  forward -> (grid [B,C,R,R,R], ind [B,N],
    norm_coords [B,3,N])."""

    def __init__(self, resolution):
        super().__init__()
        self.r = int(resolution)

    def forward(self, features, coords):
        coords = coords.detach()
        centred = coords - coords.mean(2, keepdim=True)
        radius = centred.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values
        norm_coords = centred / (radius + 1e-20)
        out, inds = F.spherical_avg_voxelize(features, norm_coords, self.r)
        return out, inds.detach(), norm_coords

    def extra_repr(self):
        return "resolution={}".format(self.r)
