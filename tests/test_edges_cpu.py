"""CPU: at BASELINE c2 scale (32 clouds x 1024 points, r = 32) every voxel
index that depends on an arithmetic choice the reference does not pin sits
on a bin edge (hard part 1):

  * FMA contraction of gamma^2 = x^2 + y^2 + z^2 (nvcc's default --fmad=true
    is the canonical choice; spherical_vox.cu:37);
  * the normalisation: the extractor's fixed-order fp64 mean / fp32 max-norm
    (oracle.normalize_sph, the kernel's order) vs the reference's torch fp32
    mean / norm / max (PVCNN/modules/spherical_vox.py:17-19), here torch on
    the CPU (tests/test_gpu_extractor.py repeats it with torch on the GPU).

The counts are printed (pytest -s) and recorded in DESIGN.md 2."""
import numpy as np
import torch

import edges
import oracle
from clouds import gaussian_clouds

B, N, R = 32, 1024, 32


def torch_normalise(xyz):
    t = torch.from_numpy(xyz)
    nc = t - t.mean(2, keepdim=True)
    nc = nc / (nc.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values + 1e-20)
    return nc.contiguous().numpy()


def test_c2_fma_sensitive_indices_are_bin_edges():
    total = explained = 0
    for seed in (0, 1):
        xyz, _, _ = gaussian_clouds(B, N, seed=seed)
        nc = oracle.normalize_sph(xyz)
        for b in range(B):
            fma = oracle.sph_index(nc[b], R, use_fma=True)
            plain = oracle.sph_index(nc[b], R, use_fma=False)
            d, e, worst = edges.explain(nc[b], nc[b], fma, plain, R)
            total += d
            explained += e
            assert d == e, "cloud %d: %d FMA-sensitive indices, %d on a bin edge (worst %.3g)" \
                % (b, d, e, worst)
    print("c2 FMA-sensitive voxel indices: %d of %d points, all on bin edges"
          % (total, 2 * B * N))
    assert total <= 2 * B * N // 1000


def test_c2_normalisation_sensitive_indices_are_bin_edges():
    total = 0
    worst_nc = 0.0
    for seed in (0, 1, 2):
        xyz, _, _ = gaussian_clouds(B, N, seed=seed)
        nc_ext = oracle.normalize_sph(xyz)
        nc_ref = torch_normalise(xyz)
        worst_nc = max(worst_nc, float(np.abs(nc_ext - nc_ref).max()))
        for b in range(B):
            a = oracle.sph_index(nc_ext[b], R)
            c = oracle.sph_index(nc_ref[b], R)
            d, e, worst = edges.explain(nc_ext[b], nc_ref[b], a, c, R)
            total += d
            assert d == e, "cloud %d: %d indices differ, %d on a bin edge (worst %.3g)" \
                % (b, d, e, worst)
    print("c2 normalisation-sensitive voxel indices (fixed-order fp64 vs torch-CPU fp32): "
          "%d of %d points; max |norm_coords diff| %.3g" % (total, 3 * B * N, worst_nc))
    assert worst_nc <= 1e-6


def _ulp_exposure(b, n, r, seeds):
    """Points whose voxel index changes when the float acos / atan of the
    voxelisation (spherical_vox.cu:46,54) return a value 1 or 2 ulps from the
    correctly rounded one (include/pcr_math.h pcr_acosf / pcr_atanf), in
    either direction, alone or both at once: (changed, explained by a bin
    edge, points)."""
    changed = explained = 0
    for seed in seeds:
        xyz, _, _ = gaussian_clouds(b, n, seed=seed)
        nc = oracle.normalize_sph(xyz)
        for i in range(b):
            base = oracle.sph_index(nc[i], r)
            assert np.array_equal(oracle.sph_index_ulp(nc[i], r, 0, 0), base)
            moved = np.zeros(n, bool)
            alt = base.copy()
            for da in range(-2, 3):
                for dt in range(-2, 3):
                    if da == 0 and dt == 0:
                        continue
                    v = oracle.sph_index_ulp(nc[i], r, da, dt)
                    new = (v != base) & ~moved
                    alt[new] = v[new]
                    moved |= v != base
            d, e, worst = edges.explain(nc[i], nc[i], base, alt, r)
            assert d == int(moved.sum())
            assert d == e, "cloud %d: %d indices move under +-2 ulp acos/atan, %d on a bin " \
                "edge (worst %.3g)" % (i, d, e, worst)
            changed += d
            explained += e
    return changed, explained, b * n * len(seeds)


def test_c2_acos_atan_ulp_exposure_is_bin_edges():
    """The 'bit-exact voxel index' claim against a real sm_61 run rests on the
    correctly rounded acos / atan here; CUDA's float overloads may be 2 ulps
    off.  At full c2 size every point whose index that could change sits on
    a bin edge; the count is the unpinned exposure."""
    d, e, pts = _ulp_exposure(B, N, R, (0, 1))
    print("c2 acos/atan +-2 ulp exposure: %d of %d points move voxel, all on bin edges"
          % (d, pts))
    assert d <= pts // 1000


def test_c5_acos_atan_ulp_exposure_is_bin_edges():
    """The same at BASELINE c5 size (8 x 65,536 points, r = 64)."""
    d, e, pts = _ulp_exposure(8, 65536, 64, (0,))
    print("c5 acos/atan +-2 ulp exposure: %d of %d points move voxel, all on bin edges"
          % (d, pts))
    assert d <= pts // 1000
