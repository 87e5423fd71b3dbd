"""PVCNN.modules mirror (reference: PVCNN/modules/__init__.py:1-10) -- the
hot-path modules.  PointNet++ set-abstraction modules, the frustum loss and
KLLoss are outside this build's scope."""
from .ball_query import BallQuery
from .knn import knnModule
from .pvconv import PVConv
from .se import SE3d
from .shared_mlp import SharedMLP
from .spherical_vox import Spherical_Voxelization
from .voxelization import Voxelization
