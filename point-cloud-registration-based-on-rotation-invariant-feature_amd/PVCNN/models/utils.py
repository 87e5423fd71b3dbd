"""Layer builders of the classifier (reference: PVCNN/models/utils.py:11-66).

Same layer sequence and module nesting as the reference, so state_dicts are
interchangeable: Linear/BN/ReLU triples (dim=1) or SharedMLP (dim=2) hidden
layers, Dropout for fractional entries, and a PVConv (or SharedMLP for a
None resolution) per block.  The PointNet++ SA/FP builders are not mirrored
(no model of the north star uses them).
"""
import functools

import torch.nn as nn

from PVCNN.modules import PVConv, SharedMLP

__all__ = ["create_mlp_components", "create_pointnet_components"]


def _linear_bn_relu(in_channels, out_channels):
    return nn.Sequential(nn.Linear(in_channels, out_channels), nn.BatchNorm1d(out_channels),
                         nn.ReLU(True))


def create_mlp_components(in_channels, out_channels, classifier=False, dim=2,
                          width_multiplier=1):
    """-> (layers, out_channels); utils.py:15-45."""
    wm = width_multiplier
    hidden = _linear_bn_relu if dim == 1 else SharedMLP
    if not isinstance(out_channels, (list, tuple)):
        out_channels = [out_channels]
    if len(out_channels) == 0 or (len(out_channels) == 1 and out_channels[0] is None):
        return nn.Sequential(), in_channels, in_channels
    layers = []
    for oc in out_channels[:-1]:
        if oc < 1:
            layers.append(nn.Dropout(oc))
            continue
        oc = int(wm * oc)
        layers.append(hidden(in_channels, oc))
        in_channels = oc
    last = out_channels[-1]
    if classifier:
        layers.append(nn.Linear(in_channels, last) if dim == 1 else
                      nn.Conv1d(in_channels, last, 1))
        return layers, last
    layers.append(_linear_bn_relu(in_channels, int(wm * last)) if dim == 1 else
                  SharedMLP(in_channels, int(wm * last)))
    return layers, int(wm * last)


def create_pointnet_components(blocks, point_kernel_formal, voxel_shape, in_channels,
                               with_coeff=False, with_se=False, normalize=True, eps=0,
                               width_multiplier=1, voxel_resolution_multiplier=1):
    """blocks = ((out_channels, num_blocks, voxel_resolution or None), ...)
    -> (layers, in_channels, concat_channels); utils.py:48-66."""
    wm, vr = width_multiplier, voxel_resolution_multiplier
    layers, concat = [], 0
    for out_channels, num_blocks, resolution in blocks:
        out_channels = int(wm * out_channels)
        if resolution is None:
            make = SharedMLP
        else:
            make = functools.partial(PVConv, point_kernel_formal=point_kernel_formal,
                                     voxel_shape=voxel_shape, kernel_size=3,
                                     resolution=int(vr * resolution), with_coeff=with_coeff,
                                     with_se=with_se, normalize=normalize, eps=eps)
        for _ in range(num_blocks):
            layers.append(make(in_channels, out_channels))
            in_channels = out_channels
            concat += out_channels
    return layers, in_channels, concat
