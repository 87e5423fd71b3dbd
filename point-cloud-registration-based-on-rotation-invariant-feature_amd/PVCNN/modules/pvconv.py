"""PVConv (reference: PVCNN/modules/pvconv.py:15-99).

Voxel branch: (spherical | cube) voxelization -> Conv3d stack (MIOpen, not
the hot path) -> devoxelization.  Point branch (dgcnn_kernel): the centre
term features - avg_grid[ind] (0 where ind == -1) is one fused gather
kernel here instead of deepcopy + gather + masked assignment.
"""
import torch
import torch.nn as nn

from . import functional as F
from .se import SE3d
from .shared_mlp import SharedMLP
from .spherical_vox import Spherical_Voxelization
from .voxelization import Voxelization
from pcr_amd import ops

__all__ = ["PVConv"]


class _CenterGather(torch.autograd.Function):
    """related = features - avg_grid[:, :, ind] (masked); gradient flows to
    features (identity on valid points) and to avg_grid (scatter of -grad)."""

    @staticmethod
    def forward(ctx, features, avg_grid, ind):
        ctx.save_for_backward(ind)
        ctx.grid_shape = avg_grid.shape
        return ops.dgcnn_center_gather(features.contiguous(), avg_grid.contiguous(),
                                       ind.contiguous())

    @staticmethod
    def backward(ctx, grad):
        (ind,) = ctx.saved_tensors
        valid = (ind != -1).unsqueeze(1).to(grad.dtype)
        g_feat = grad * valid
        g_grid = torch.zeros(ctx.grid_shape, dtype=grad.dtype, device=grad.device)
        idx = ind.clamp(min=0).long().unsqueeze(1).expand(-1, grad.shape[1], -1)
        g_grid.scatter_add_(2, idx, -g_feat)
        return g_feat, g_grid, None


class PVConv(nn.Module):
    def __init__(self, in_channels, out_channels, point_kernel_formal, voxel_shape, kernel_size,
                 resolution, with_coeff=False, with_se=False, normalize=True, eps=0):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.point_kernel_formal = point_kernel_formal
        self.kernel_size = kernel_size
        self.resolution = resolution
        self.voxel_shape = voxel_shape
        self.with_coeff = with_coeff
        self.voxelization = Voxelization(resolution, normalize=normalize, eps=eps)
        self.spherical_vox = Spherical_Voxelization(resolution)
        if with_coeff:
            self.coefficient = nn.Parameter(torch.Tensor([1]))
        pad = kernel_size // 2
        layers = [
            nn.Conv3d(in_channels, out_channels, kernel_size, stride=1, padding=pad),
            nn.BatchNorm3d(out_channels, eps=1e-4),
            nn.LeakyReLU(0.1, True),
            nn.Conv3d(out_channels, out_channels, kernel_size, stride=1, padding=pad),
            nn.BatchNorm3d(out_channels, eps=1e-4),
            nn.LeakyReLU(0.1, True),
        ]
        if with_se:
            layers.append(SE3d(out_channels))
        self.voxel_layers = nn.Sequential(*layers)
        mlp_in = in_channels * 2 if point_kernel_formal == "dgcnn_kernel" else in_channels
        self.point_layers = SharedMLP(mlp_in, out_channels)

    def forward(self, inputs):
        features, coords = inputs
        b, c, n = features.shape
        if self.voxel_shape == "cube":
            avg, inds, vcoords = self.voxelization(features, coords)
            vox = F.trilinear_devoxelize(self.voxel_layers(avg), vcoords, self.resolution,
                                         self.training)
        elif self.voxel_shape == "spherical":
            avg, inds, vcoords = self.spherical_vox(features, coords)
            vox = F.spherical_trilinear_devoxelize(self.voxel_layers(avg), vcoords, inds,
                                                   self.resolution, self.training)
        else:
            raise ValueError("voxel_shape must be 'cube' or 'spherical'")
        if self.point_kernel_formal == "dgcnn_kernel":
            related = _CenterGather.apply(features, avg.view(b, c, -1), inds.to(torch.int32))
            point = self.point_layers(torch.cat((related, features), 1))
        elif self.point_kernel_formal == "pointnet_kernel":
            point = self.point_layers(features)
        else:
            raise ValueError("unknown point_kernel_formal %r" % self.point_kernel_formal)
        fused = self.coefficient * vox + point if self.with_coeff else vox + point
        return fused, coords
