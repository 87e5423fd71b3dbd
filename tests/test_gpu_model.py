"""The sph-dg / cu-dg PVCNN_classifier (PVCNN/models/pvcnn_classify.py:14-345)
on the MI355X path against a torch fp32 restatement of the reference forward
(tests/model_restate.py): same weights, forward + backward, at the c3
per-cloud shape (N = 2048 points) with a small batch.

Tolerances: the two forwards differ only in fp32 summation order (voxel
means, devox sums, local-PPF acos within 1e-5) and in the atomic order of
the backward scatters, amplified through four blocks of Conv3d + BatchNorm;
the logits must agree to 1e-3 and every parameter gradient to 3e-3
relative (norm-wise; the with_coeff scalar sums ~1e5 products with
cancellation), far below anything a wrong index or corner would give.
"""
import numpy as np
import pytest
import torch

from clouds import gaussian_clouds
from model_restate import classifier_forward_torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def full_fp32_convs():
    """The Conv3d / Conv1d / Linear layers both forwards share run in full
    fp32: with TF32-style reduced-precision convolutions allowed (PyTorch's
    default for cudnn/MIOpen), the library may pick a different algorithm
    for the second of two identical calls and the two forwards then differ
    by ~1e-2 -- noise that has nothing to do with the hot path."""
    saved = (torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32,
             torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    yield
    (torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32,
     torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark) = saved

# configs/modelnet40/pvcnn/__init__.py:5-8
DIM_K = 512
BLOCKS = ((64, 1, 32), (128, 1, 32), (256, 1, None), (DIM_K, 1, None))


def sph_dg(**kw):
    """configs/modelnet40/pvcnn/experiments/SO3_SO3/exp13.py"""
    from PVCNN.models.pvcnn_classify import PVCNN_classifier
    args = dict(blocks=BLOCKS, dim_k=DIM_K, point_kernel_formal="dgcnn_kernel",
                voxel_shape="spherical", num_classes=40, extra_feature_channels=0,
                rot_invariant_preprocess="change_coords", with_local_feat="ppf",
                with_transform_fine_tune=False, use_new_coords_for_voxel=False,
                with_coeff=True, with_se=True)
    args.update(kw)
    return PVCNN_classifier(**args)


def cu_dg(**kw):
    """configs/.../SO3_SO3/deepgmr_mn40_cu_dg/__init__.py (registration
    features: is_classify False, extra_feature_channels 4)."""
    args = dict(voxel_shape="cube", extra_feature_channels=4, with_coeff=False,
                is_classify=False)
    args.update(kw)
    return sph_dg(**args)


def inputs_for(b, n, seed):
    xyz, nrm, _ = gaussian_clouds(b, n, seed=seed)
    xyz = xyz * 0.35  # ModelNet40-like extent, so the r = 0.3 ball holds tens of points
    return torch.from_numpy(np.concatenate([xyz, nrm], axis=1)).float()


def rel_err(a, b):
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def bn_fed_biases(model):
    """Names of the conv / linear biases whose output goes straight into a
    BatchNorm: their exact gradient is 0 (BN subtracts the batch mean), so
    both sides hold only rounding noise there."""
    names = set()
    for prefix, mod in model.named_modules():
        if isinstance(mod, torch.nn.Sequential):
            kids = list(mod.named_children())
            for (na, a), (_, nb) in zip(kids, kids[1:]):
                if isinstance(nb, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d,
                                   torch.nn.BatchNorm3d)) and getattr(a, "bias", None) is not None:
                    names.add("%s.%s.bias" % (prefix, na) if prefix else "%s.bias" % na)
    return names


def _check_model(model, x):
    dev = x.device
    model = model.to(dev).train()
    # the classifier's BatchNorm1d over a batch of 2 would normalise each
    # feature to +-1 and leave only cancellation noise in every upstream
    # gradient: run it (and its dropout) on running statistics instead
    model.classifier.eval()
    torch.manual_seed(0)
    out = model(x)
    loss = (out * torch.linspace(-1, 1, out.numel(), device=dev).view_as(out)).sum()
    loss.backward()
    g_mine = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad()
    torch.manual_seed(0)
    ref = classifier_forward_torch(model, x)
    lref = (ref * torch.linspace(-1, 1, ref.numel(), device=dev).view_as(ref)).sum()
    lref.backward()
    g_ref = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    assert out.shape == ref.shape
    assert torch.isfinite(out).all()
    assert rel_err(out.detach(), ref.detach()) < 1e-3, rel_err(out.detach(), ref.detach())
    assert set(g_mine) == set(g_ref)
    noise = {k for k in bn_fed_biases(model) if k in g_mine and not k.startswith("classifier.")}
    assert noise, "expected BN-fed biases"
    for k in noise:
        w = k[:-len("bias")] + "weight"
        assert g_mine[k].norm() <= 1e-3 * g_mine[w].norm(), k
    worst = max((k for k in g_mine if k not in noise), key=lambda k: rel_err(g_mine[k], g_ref[k]))
    assert rel_err(g_mine[worst], g_ref[worst]) < 3e-3, (worst, rel_err(g_mine[worst],
                                                                         g_ref[worst]))
    return out


def test_sph_dg_forward_backward(dev):
    x = inputs_for(2, 2048, seed=21).to(dev)
    out = _check_model(sph_dg(), x)
    assert out.shape == (2, 40)


def test_cu_dg_forward_backward(dev):
    x = inputs_for(2, 2048, seed=22).to(dev)
    out = _check_model(cu_dg(), x)
    assert out.shape == (2, DIM_K, 2048)


def test_ppf_preprocess_model(dev):
    """rot_invariant_preprocess == 'ppf' (global PPF kernel, :99-117)."""
    x = inputs_for(2, 1024, seed=23).to(dev)
    out = _check_model(sph_dg(rot_invariant_preprocess="ppf", extra_feature_channels=3), x)
    assert out.shape == (2, 40)


def test_local_ppf_fused_equals_composition(dev):
    """The fused ball-query + local-PPF path equals the reference's
    differentiable composition (BallQuery grouping + torch math) run on the
    same kernels: |d| within 1 ulp, angles within the north-star 1e-5 --
    except where the cosine is so close to +-1 that acos turns a 1-ulp
    difference of the two dot products (fused fmaf chain vs torch's
    mul + sum, after du = d / |d| already differs by an ulp per component)
    into more than 1e-5; there the cosines agree within 8 ulps."""
    model = sph_dg().to(dev)
    x = inputs_for(2, 2048, seed=24).to(dev)
    coords = x[:, :3] - x[:, :3].mean(dim=2, keepdim=True)
    with torch.no_grad():
        fused = model._local_ppf(coords, x[:, 3:6])
    c2 = coords.clone().requires_grad_(True)
    comp = model._local_ppf(c2, x[:, 3:6])
    assert fused.shape == comp.shape == (2, 4, 128, 2048)
    finite = torch.isfinite(comp)
    assert torch.equal(finite, torch.isfinite(fused))
    comp = comp.detach()
    ok = finite.all(dim=1, keepdim=True).expand_as(comp)
    dn_f, dn_c = fused[:, 3][ok[:, 3]], comp[:, 3][ok[:, 3]]
    dn_rel = ((dn_f - dn_c).abs() / dn_c.abs()).max().item()
    assert dn_rel <= 2.4e-7, dn_rel  # 2 ulp: fmaf chain vs torch.norm's order
    af, ac = fused[:, :3][ok[:, :3]], comp[:, :3][ok[:, :3]]
    close_angle = (af - ac).abs() <= 1e-5
    close_cos = (torch.cos(af.double()) - torch.cos(ac.double())).abs() <= 8 * 2.0 ** -24
    bad = ~(close_angle | close_cos)
    assert not bad.any(), (af[bad][:5], ac[bad][:5])
    assert close_angle.float().mean() > 0.999, close_angle.float().mean()
