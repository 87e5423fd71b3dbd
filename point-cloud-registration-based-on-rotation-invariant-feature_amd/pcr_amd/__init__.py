"""pcr_amd -- MI355X (gfx950) hot path of the rotation-invariant point-cloud
registration network: KNN / ball-query neighbour search, point-pair features,
spherical and cube voxelize/devoxelize, as hand-written HIP kernels behind the
C ABI of libpcr_amd.so (include/pcr_amd.h).

``pcr_amd.ops`` mirrors the reference's ``_backend`` functions on torch
tensors; ``PVCNN`` (a sibling package) mirrors the reference's
``PVCNN.modules.functional`` / ``PVCNN.modules`` Python API on top of it;
``pcr_amd.extractor`` is the fused sph-dg extractor forward used by bench.py;
``pcr_amd.distributed`` shards batches over ranks and all-gathers descriptors.
"""
from . import _lib  # noqa: F401
from ._lib import load, version  # noqa: F401

__all__ = ["load", "version", "ops", "extractor", "distributed"]
