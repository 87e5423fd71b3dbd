"""SharedMLP (reference: PVCNN/modules/shared_mlp.py:6-36): 1x1 conv + BN + ReLU
stack.  Plain torch (MIOpen); outside the hot path, present so PVConv and the
models import unchanged."""
import torch.nn as nn

__all__ = ["SharedMLP"]


class SharedMLP(nn.Module):
    def __init__(self, in_channels, out_channels, dim=1):
        super().__init__()
        conv, bn = {1: (nn.Conv1d, nn.BatchNorm1d), 2: (nn.Conv2d, nn.BatchNorm2d)}[dim]
        if not isinstance(out_channels, (list, tuple)):
            out_channels = [out_channels]
        layers = []
        for oc in out_channels:
            if oc < 1:
                layers.append(nn.Dropout(oc))
                continue
            layers += [conv(in_channels, oc, 1), bn(oc), nn.ReLU(True)]
            in_channels = oc
        self.layers = nn.Sequential(*layers)

    def forward(self, inputs):
        if isinstance(inputs, (list, tuple)):
            return (self.layers(inputs[0]), *inputs[1:])
        return self.layers(inputs)
