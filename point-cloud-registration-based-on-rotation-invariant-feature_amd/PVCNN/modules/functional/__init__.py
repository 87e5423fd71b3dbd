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
from .interpolatation import nearest_neighbor_interpolate
from .sampling import gather, furthest_point_sample, logits_mask
from .loss import kl_loss, huber_loss
from .lrf import change_coords
