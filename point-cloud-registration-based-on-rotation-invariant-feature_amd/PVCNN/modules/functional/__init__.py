"""PVCNN.modules.functional mirror (reference: PVCNN/modules/functional/__init__.py:1-11)."""
from .ball_query import ball_query
from .devoxelization import trilinear_devoxelize
from .grouping import grouping
from .voxelization import avg_voxelize
from .spherical_vox import spherical_avg_voxelize
from .spherical_devox import spherical_trilinear_devoxelize
from .ppf import ppf
from .knn import k_nearest_neighbor
from .local_ppf import local_ppf, knn_local_ppf
from pcr_amd.ops import _out_of_scope

# PointNet++ helpers of the reference package (unused by the sph-dg / cu-dg
# configs) -- present as names, raise when called.
nearest_neighbor_interpolate = _out_of_scope("nearest_neighbor_interpolate")
gather = _out_of_scope("gather")
furthest_point_sample = _out_of_scope("furthest_point_sample")
logits_mask = _out_of_scope("logits_mask")
kl_loss = _out_of_scope("kl_loss")
huber_loss = _out_of_scope("huber_loss")
