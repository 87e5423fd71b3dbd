"""Drop-in mirror of the reference's ``PVCNN`` package path for the hot path.

Put ``point-cloud-registration-based-on-rotation-invariant-feature_amd/`` on
``sys.path`` and ``import PVCNN.modules.functional as F`` /
``from PVCNN.modules import PVConv, Spherical_Voxelization, ...`` resolve to
the MI355X implementation with the reference's signatures.
"""
