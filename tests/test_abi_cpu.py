"""CPU: the C-ABI library builds, loads, and exports every symbol the header
declares; the Python mirror imports with the reference's names."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pcr_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pcr_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    from pcr_amd import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, "ctypes signature missing for %s" % s
    assert set(_lib.SIGNATURES) == set(syms)
    assert "gfx950" in _lib.version()


def test_library_is_gfx950_code_object():
    from pcr_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle target id
    assert b"vox_grid_kernel" in data and b"knn_kernel" in data
    assert b"fps_reg_kernel" in data and b"lrf_kernel" in data and b"three_nn_kernel" in data


def test_backend_names_match_reference_bindings():
    from PVCNN.modules.functional.backend import _backend
    # src/bindings.cpp:14-55
    for name in ["gather_features_forward", "gather_features_backward", "furthest_point_sampling",
                 "ball_query", "grouping_forward", "grouping_backward",
                 "three_nearest_neighbors_interpolate_forward",
                 "three_nearest_neighbors_interpolate_backward", "trilinear_devoxelize_forward",
                 "trilinear_devoxelize_backward", "avg_voxelize_forward", "avg_voxelize_backward",
                 "spherical_avg_voxelize_forward", "spherical_avg_voxelize_backward",
                 "spherical_trilinear_devoxelize_forward",
                 "spherical_trilinear_devoxelize_backward", "spherical_ppf_forward",
                 "knn_forward_cuda", "knn_backward_cuda"]:
        assert callable(getattr(_backend, name)), name


def test_python_api_surface():
    import PVCNN.modules.functional as F
    from PVCNN.modules import (BallQuery, PVConv, SE3d, SharedMLP, Spherical_Voxelization,
                               Voxelization, knnModule)
    for name in ["ball_query", "trilinear_devoxelize", "grouping", "avg_voxelize",
                 "spherical_avg_voxelize", "spherical_trilinear_devoxelize", "ppf",
                 "k_nearest_neighbor", "nearest_neighbor_interpolate", "gather",
                 "furthest_point_sample", "logits_mask", "kl_loss", "huber_loss",
                 "change_coords"]:
        assert hasattr(F, name), name
    del BallQuery, PVConv, SE3d, SharedMLP, Spherical_Voxelization, Voxelization, knnModule


def test_cpu_tensors_rejected_like_reference():
    torch = pytest.importorskip("torch")
    from pcr_amd import ops
    x = torch.zeros((1, 3, 8))
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ops.spherical_avg_voxelize_forward(x, x, 4)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ops.knn_forward_cuda(x, x, 2)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ops.furthest_point_sampling(x, 4)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ops.three_nearest_neighbors_interpolate_forward(x, x, x)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ops.lrf_change_coords(x)


def test_workspace_size_query():
    from pcr_amd import _lib
    lib = _lib.load()
    assert lib.pcr_voxelize_workspace_size(32, 1024, 32) > 32 * 1024 * 4 * 3
    assert lib.pcr_voxelize_workspace_size(0, 0, 0) == 256


def test_extractor_structs_match_header(tmp_path):
    """The ctypes mirrors of pcr_extractor_args / pcr_extractor_set
    (pcr_amd/_lib.py) have the header's size and field offsets (gcc on the
    header; a mismatch would hand the runner garbage pointers)."""
    import ctypes
    import subprocess
    from pcr_amd import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pcr_amd.h"',
             'int main(void) {']
    for cname, cls in (("pcr_extractor_args", _lib.ExtractorArgs),
                       ("pcr_extractor_set", _lib.ExtractorSet)):
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines += ['return 0;', '}']
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = subprocess.check_output([str(exe)]).decode().split("\n")
    want = []
    for cname, cls in (("pcr_extractor_args", _lib.ExtractorArgs),
                       ("pcr_extractor_set", _lib.ExtractorSet)):
        want.append("%s size %d" % (cname, ctypes.sizeof(cls)))
        want += ["%s %s %d" % (cname, f[0], getattr(cls, f[0]).offset) for f in cls._fields_]
    assert [g for g in got if g] == want
