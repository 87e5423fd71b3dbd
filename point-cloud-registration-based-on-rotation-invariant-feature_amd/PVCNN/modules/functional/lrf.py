"""change_coords: the local-reference-frame preprocessing of the reference
model (PVCNN/models/pvcnn_classify.py:153-184, rot_invariant_preprocess ==
'change_coords'), one GPU launch for the whole batch in place of the
reference's per-cloud Python loop."""
from pcr_amd import ops

__all__ = ["change_coords"]


def change_coords(coords, check=True):
    """coords [B,3,N] -> new_coords [B,3,N]: each cloud centred and expressed
    in the frame (base_x, base_y, base_z).  base_x is the farthest point from
    the centroid.  base_y is the next point in descending-norm order whose
    direction is not within |cos| >= 0.9 of base_x.  Then Gram-Schmidt and a
    cross product.  Raises AssertionError where the reference's asserts
    would (:159, :169, :177).  No autograd: the reference computes the frame
    from detached indices too."""
    return ops.lrf_change_coords(coords.contiguous(), check=check)
