"""SE3d (reference: PVCNN/modules/se.py:6-17): squeeze-excitation over a voxel
grid.  Plain torch; outside the hot path."""
import torch.nn as nn

__all__ = ["SE3d"]


class SE3d(nn.Module):
    def __init__(self, channel, reduction=8):
        super().__init__()
        hidden = channel // reduction
        self.fc = nn.Sequential(nn.Linear(channel, hidden, bias=False), nn.ReLU(inplace=True),
                                nn.Linear(hidden, channel, bias=False), nn.Sigmoid())

    def forward(self, inputs):
        w = self.fc(inputs.mean(dim=(2, 3, 4)))
        return inputs * w.view(inputs.shape[0], inputs.shape[1], 1, 1, 1)
