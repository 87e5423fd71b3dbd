"""ctypes binding of libpcr_amd.so (the C ABI declared in include/pcr_amd.h).

This is the reference-side binding a maintainer adds to call the MI355X
library: every symbol of the header with its exact C signature.  There is no
CPU fallback anywhere in the product path -- if the shared library is missing
or a call fails, a RuntimeError is raised.
"""
import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("PCR_AMD_LIB", os.path.join(_PKG_ROOT, "lib", "libpcr_amd.so"))
CSRC_DIR = os.path.join(_PKG_ROOT, "csrc")

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
SZ = ctypes.c_size_t
ST = ctypes.c_int

# name -> (restype, argtypes); mirrors include/pcr_amd.h one to one
SIGNATURES = {
    "pcr_last_error": (ctypes.c_char_p, []),
    "pcr_version": (ctypes.c_char_p, []),
    "pcr_stream_create_cu_mask": (ST, [P, I, ctypes.POINTER(P)]),
    "pcr_stream_destroy": (ST, [P]),
    "pcr_knn_forward": (ST, [P, P, I, I, I, I, I, P, P, P, P, P, SZ, P]),
    "pcr_knn_workspace_size": (SZ, [I, I, I]),
    "pcr_knn_backward": (ST, [P, P, P, P, P, P, I, I, I, I, I, P, P, P]),
    "pcr_knn_backward_workspace_size": (SZ, [I, I, I, I]),
    "pcr_knn_backward_ws": (ST, [P, P, P, P, P, P, I, I, I, I, I, P, P, P, SZ, P]),
    "pcr_spherical_ppf_forward": (ST, [P, P, P, P, I, I, P, P]),
    "pcr_local_ppf_forward": (ST, [P, P, P, P, P, I, I, I, I, I, I, P, P]),
    "pcr_knn_local_ppf": (ST, [P, P, I, I, I, I, P, P, P, P, SZ, P]),
    "pcr_knn_prepare": (ST, [P, I, I, P, SZ, P]),
    "pcr_knn_local_ppf_prepared": (ST, [P, P, I, I, I, I, P, P, P, P, SZ, P]),
    "pcr_knn_select_ppf": (ST, [P, P, I, I, I, I, P, P, P, SZ, P]),
    "pcr_knn_select_sorted": (ST, [P, I, I, I, P, SZ, P]),
    "pcr_knn_ppf_sorted": (ST, [P, P, I, I, I, I, P, P, P, SZ, P]),
    "pcr_ball_query": (ST, [P, P, I, I, I, F, I, P, P]),
    "pcr_grouping_forward": (ST, [P, P, I, I, I, I, I, P, P]),
    "pcr_grouping_backward": (ST, [P, P, I, I, I, I, I, P, P]),
    "pcr_voxelize_workspace_size": (SZ, [I, I, I]),
    "pcr_voxelize_workspace_size_c": (SZ, [I, I, I, I]),
    "pcr_spherical_avg_voxelize_forward": (ST, [P, P, I, I, I, I, P, P, P, P, SZ, P]),
    "pcr_avg_voxelize_forward": (ST, [P, P, I, I, I, I, P, P, P, P, SZ, P]),
    "pcr_avg_voxelize_backward": (ST, [P, P, P, I, I, I, I, P, P]),
    "pcr_spherical_normalize": (ST, [P, I, I, P, P]),
    "pcr_spherical_trilinear_devoxelize_forward": (ST, [I, I, P, P, P, I, I, I, P, P, P, P]),
    "pcr_trilinear_devoxelize_forward": (ST, [I, I, P, P, I, I, I, P, P, P, P]),
    "pcr_devoxelize_backward": (ST, [P, P, P, I, I, I, I, I, P, P]),
    "pcr_devoxelize_backward_workspace_size": (SZ, [I, I]),
    "pcr_devoxelize_backward_workspace_size_r": (SZ, [I, I, I, I]),
    "pcr_devoxelize_backward_ws": (ST, [P, P, P, I, I, I, I, I, P, P, SZ, P]),
    "pcr_dgcnn_center_gather": (ST, [P, P, P, I, I, I, I, P, P]),
    "pcr_extractor_workspace_size": (SZ, [I, I, I, I]),
    "pcr_extractor_voxel_stage": (ST, [P, P, I, I, I, I, P, P, P, P, P, P, P, P, P, SZ, P]),
    "pcr_extractor_voxel_prep": (ST, [P, I, I, I, P, P, P, P, P, SZ, P]),
    "pcr_extractor_voxel_grid": (ST, [P, I, I, I, I, P, P, P, SZ, P]),
    "pcr_extractor_voxel_devox": (ST, [P, I, I, I, I, P, P, P, P, P, SZ, P]),
    "pcr_extractor_grid_devox": (ST, [P, P, P, I, I, I, I, P, P, P]),
    "pcr_extractor_voxel_grid_devox": (ST, [P, I, I, I, I, P, P, P, P, P, P, P, SZ, P]),
    "pcr_extractor_voxel_means_devox": (ST, [P, I, I, I, I, P, P, P, P, P, SZ, P]),
    "pcr_extractor_voxel_stream": (ST, [I, I, I, I, P, P, P, SZ, P]),
    "pcr_extractor_stream_devox_ok": (I, [I, I, I]),
    "pcr_extractor_voxel_means": (ST, [P, I, I, I, I, P, SZ, P]),
    "pcr_extractor_voxel_stream_devox": (ST, [I, I, I, I, P, P, P, P, P, P, SZ, P]),
    "pcr_runner_create": (ST, [I, ctypes.POINTER(P)]),
    "pcr_runner_destroy": (None, [P]),
    "pcr_runner_grid_times": (ST, [P, P, I, ctypes.POINTER(I)]),
    "pcr_runner_set_timed": (ST, [P, I]),
    "pcr_extractor_run": (ST, [P, P, I, I, P, P, P, P, P]),
    "pcr_mutual_nn_workspace_size": (SZ, [I, I, I]),
    "pcr_mutual_nn_match": (ST, [P, P, I, I, I, I, P, P, P, P, P, P, SZ, P]),
    "pcr_mutual_nn_match_cm": (ST, [P, P, I, I, I, I, P, P, P, P, P, P, SZ, P]),
    "pcr_lrf_change_coords": (ST, [P, I, I, P, P, P, P, P]),
    "pcr_gather_features_forward": (ST, [P, P, I, I, I, I, P, P]),
    "pcr_gather_features_backward": (ST, [P, P, I, I, I, I, P, P]),
    "pcr_fps_workspace_size": (SZ, [I, I]),
    "pcr_furthest_point_sampling": (ST, [P, I, I, I, P, P, SZ, P]),
    "pcr_three_nn_interpolate_forward": (ST, [P, P, P, I, I, I, I, P, P, P, P]),
    "pcr_three_nn_interpolate_backward": (ST, [P, P, P, I, I, I, I, P, P]),
    "pcr_estimate_normals": (ST, [P, I, I, ctypes.c_double, P, P, P]),
    "pcr_txt_shape": (ST, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong),
                           ctypes.POINTER(ctypes.c_int)]),
    "pcr_read_xyzn_txt": (ST, [ctypes.c_char_p, P, ctypes.c_longlong, I]),
    "pcr_selftest_math": (ST, [I, P, P, I, I, P, P, P]),
    "pcr_selftest_math_d": (ST, [I, P, P, I, P, P]),
}



class ExtractorSet(ctypes.Structure):
    """struct pcr_extractor_set of include/pcr_amd.h (one batch-ring set)"""
    _fields_ = [("xyz", P), ("normals", P), ("features", P), ("knn_idx", P), ("knn_dist", P),
                ("local_ppf", P), ("norm_coords", P), ("ind", P), ("cnt", P), ("grid", P),
                ("devox", P), ("desc", P), ("dinds", P), ("dwgts", P), ("corr12", P),
                ("corr21", P), ("idx1", P), ("idx2", P), ("match_count", P)]


class ExtractorArgs(ctypes.Structure):
    """struct pcr_extractor_args of include/pcr_amd.h"""
    _fields_ = [("b", I), ("n", I), ("c", I), ("k", I), ("r", I), ("relative", I),
                ("xyz", P), ("normals", P), ("features", P), ("knn_idx", P), ("knn_dist", P),
                ("local_ppf", P), ("norm_coords", P), ("ind", P), ("cnt", P), ("grid", P),
                ("devox", P), ("desc", P), ("dinds", P * 2), ("dwgts", P * 2), ("knn_ws", P * 2),
                ("knn_ws_bytes", SZ), ("vox_ws", P * 2), ("vox_ws_bytes", SZ),
                ("match_pairs", I), ("corr12", P), ("corr21", P), ("idx1", P), ("idx2", P),
                ("match_count", P), ("match_ws", P), ("match_ws_bytes", SZ),
                ("nsets", I), ("set0", I), ("sets", ctypes.POINTER(ExtractorSet)),
                ("vox_ws3", P), ("devox_in_means", I)]


_lib = None


def load():
    """Load libpcr_amd.so once; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            "libpcr_amd.so not found at %s -- build it with `make -C %s` "
            "(or __graft_entry__.build()); there is no CPU fallback" % (LIB_PATH, CSRC_DIR))
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status, what):
    if status != 0:
        msg = load().pcr_last_error()
        raise RuntimeError("%s failed (status %d): %s" % (what, status, msg.decode() if msg else ""))


def version():
    return load().pcr_version().decode()
