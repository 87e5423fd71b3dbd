"""Local k-neighbour PPF of the sph-dg model as one fused op.

Reference: PVCNN/models/pvcnn_classify.py:252-269 (BallQuery(0.3, 128)
grouping of coords and normals, d = c - grouped_rel, three acos and |d|),
done there with ~10 separate torch kernels and [B,3,U,N] intermediates.
"""
import torch

from pcr_amd import ops

__all__ = ["local_ppf", "knn_local_ppf"]


def local_ppf(coords, normals, neighbor_indices, relative=True):
    """coords/normals [B,3,N] (centres == points, as in the model),
    neighbor_indices [B,N,U] from ball_query -> local PPF [B,4,U,N]
    (nr_d, ni_d, nr_ni, |d|)."""
    coords = coords.contiguous()
    normals = normals.contiguous()
    return ops.local_ppf_forward(coords, normals, coords, normals,
                                 neighbor_indices.to(torch.int32).contiguous(), kmajor=False,
                                 relative=relative)


def knn_local_ppf(coords, normals, k, relative=True):
    """Self-KNN (k, self included) + local PPF in one kernel ->
    (idx [B,k,N], local PPF [B,4,k,N])."""
    idx, ppf, _ = ops.knn_local_ppf(coords.contiguous(), normals.contiguous(), k, relative)
    return idx, ppf
