"""knnModule (reference: PVCNN/modules/knn.py:4-26)."""
import torch.nn as nn

from .functional.knn import k_nearest_neighbor

__all__ = ["knnModule"]


class knnModule(nn.Module):
    """forward(input1, input2, k, bilateral, return_distance, return_index):
    distances are returned as sqrt of the squared KNN distances."""

    def forward(self, input1, input2, k, bilateral, return_distance, return_index):
        dist1, dist2, idx1, idx2 = k_nearest_neighbor(input1, input2, k)
        out = []
        if return_distance:
            out.append(dist1.sqrt())
            if bilateral:
                out.append(dist2.sqrt())
        if return_index:
            out.append(idx1)
            if bilateral:
                out.append(idx2)
        if not out:
            return None
        if return_distance and return_index:
            # reference order: (d1[, d2], i1[, i2])
            return tuple(out)
        return out[0] if len(out) == 1 else tuple(out)
