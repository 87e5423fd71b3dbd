"""PVCNN.models mirror (reference: PVCNN/models/__init__.py).

``from PVCNN.models.pvcnn_classify import PVCNN_classifier`` -- the import
line of configs/modelnet40/pvcnn/__init__.py:1 -- resolves here.  The
PointNet / PointNet++ baselines (models/pointnet*.py) are outside the hot
path and not mirrored.
"""
from . import pvcnn_classify, utils  # noqa: F401
