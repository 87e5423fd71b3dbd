"""BallQuery (reference: PVCNN/modules/ball_query.py:9-39)."""
import torch
import torch.nn as nn

from . import functional as F

__all__ = ["BallQuery"]


class BallQuery(nn.Module):
    """forward(points_coords, centers_coords, points_features=None) ->
    [B, 3(+C), U, M]: neighbour coordinates RELATIVE to their centre (the
    source of the model's d = 2c - p local-PPF quirk) concatenated with the
    grouped features."""

    def __init__(self, radius, num_neighbors, include_coordinates=True):
        super().__init__()
        self.radius = radius
        self.num_neighbors = num_neighbors
        self.include_coordinates = include_coordinates

    def forward(self, points_coords, centers_coords, points_features=None):
        points_coords = points_coords.contiguous()
        centers_coords = centers_coords.contiguous()
        idx = F.ball_query(centers_coords, points_coords, self.radius, self.num_neighbors)
        rel = F.grouping(points_coords, idx) - centers_coords.unsqueeze(-1)
        if points_features is None:
            assert self.include_coordinates, "No Features For Grouping"
            grouped = rel
        else:
            grouped = F.grouping(points_features, idx)
            if self.include_coordinates:
                grouped = torch.cat([rel, grouped], dim=1)
        return grouped.permute(0, 1, 3, 2)

    def extra_repr(self):
        return "radius={}, num_neighbors={}{}".format(
            self.radius, self.num_neighbors, ", include coordinates" if self.include_coordinates else "")
