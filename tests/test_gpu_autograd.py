"""GPU: the reference-compatible autograd / nn.Module layer (PVCNN mirror)
against plain PyTorch fp32 restatements of the same ops."""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_spherical_voxelization_module_grad(dev):
    import PVCNN.modules.functional as F
    from PVCNN.modules import Spherical_Voxelization
    b, n, c, r = 2, 1024, 8, 16
    xyz, _, feat = gaussian_clouds(b, n, seed=2, c=c)
    tf = T(feat, dev).requires_grad_(True)
    vox = Spherical_Voxelization(r)
    out, ind, nc = vox(tf, T(xyz, dev))
    assert out.shape == (b, c, r, r, r) and ind.shape == (b, n)
    # torch fp32 restatement of the scatter-mean
    indl = ind.long()
    valid = indl >= 0
    cnt = torch.zeros((b, r ** 3), device=dev)
    ref = torch.zeros((b, c, r ** 3), device=dev)
    for bi in range(b):
        cnt[bi].index_add_(0, indl[bi][valid[bi]], torch.ones(int(valid[bi].sum()), device=dev))
    inv = torch.where(cnt > 0, 1.0 / cnt.clamp(min=1), torch.zeros_like(cnt))
    tf2 = tf.detach().clone().requires_grad_(True)
    for bi in range(b):
        w = inv[bi][indl[bi].clamp(min=0)] * valid[bi]
        ref[bi] = ref[bi].index_add(1, indl[bi].clamp(min=0), tf2[bi] * w)
    assert torch.allclose(out.view(b, c, -1), ref, atol=1e-5)
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go.view(b, c, -1))
    assert torch.allclose(tf.grad, tf2.grad, atol=1e-5)
    del F


def test_spherical_devox_grad(dev):
    import PVCNN.modules.functional as F
    b, n, c, r = 2, 512, 4, 16
    xyz, _, feat = gaussian_clouds(b, n, seed=4, c=c)
    nc = oracle.normalize_sph(xyz)
    _, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    grid = T(np.random.default_rng(1).standard_normal((b, c, r, r, r)).astype(np.float32), dev)
    grid.requires_grad_(True)
    out = F.spherical_trilinear_devoxelize(grid, T(nc, dev), T(ind, dev), r, True)
    _, inds, wgts = oracle.spherical_trilinear_devoxelize_forward(r, nc, N(grid.view(b, c, -1)),
                                                                  ind)
    # torch restatement: out = sum_q w_q * grid[inds_q]
    ti, tw = T(inds, dev).long(), T(wgts, dev)
    g2 = grid.detach().clone().view(b, c, -1).requires_grad_(True)
    ref = torch.zeros((b, c, n), device=dev)
    skip = ti[:, 0, :] == -1
    for q in range(8):
        idx = ti[:, q, :].clamp(min=0).unsqueeze(1).expand(-1, c, -1)
        ref = ref + tw[:, q, :].unsqueeze(1) * torch.gather(g2, 2, idx) * (~skip).unsqueeze(1)
    assert torch.allclose(out, ref, atol=1e-5)
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go)
    assert torch.allclose(grid.grad.view(b, c, -1), g2.grad, atol=1e-4)


def N(t):
    return t.detach().cpu().numpy()


def test_knn_module_and_grad(dev):
    from PVCNN.modules import knnModule
    from PVCNN.modules.functional import k_nearest_neighbor
    rng = np.random.default_rng(0)
    x1 = T(rng.standard_normal((2, 3, 200)).astype(np.float32), dev).requires_grad_(True)
    x2 = T(rng.standard_normal((2, 3, 150)).astype(np.float32), dev).requires_grad_(True)
    d1, d2, i1, i2 = k_nearest_neighbor(x1, x2, 8)
    (d1.sum() + 2 * d2.sum()).backward()
    # torch restatement of the distances and their gradient
    y1 = x1.detach().clone().requires_grad_(True)
    y2 = x2.detach().clone().requires_grad_(True)
    g1 = torch.gather(y2.unsqueeze(2).expand(-1, -1, 8, -1), 3,
                      i1.long().unsqueeze(1).expand(-1, 3, -1, -1))
    r1 = ((y1.unsqueeze(2) - g1) ** 2).sum(1)
    g2 = torch.gather(y1.unsqueeze(2).expand(-1, -1, 8, -1), 3,
                      i2.long().unsqueeze(1).expand(-1, 3, -1, -1))
    r2 = ((y2.unsqueeze(2) - g2) ** 2).sum(1)
    assert torch.allclose(r1, d1, atol=1e-5) and torch.allclose(r2, d2, atol=1e-5)
    (r1.sum() + 2 * r2.sum()).backward()
    assert torch.allclose(x1.grad, y1.grad, atol=1e-4)
    assert torch.allclose(x2.grad, y2.grad, atol=1e-4)
    dist, idx = knnModule()(x1, x2, 8, False, True, True)
    assert torch.allclose(dist, d1.sqrt()) and torch.equal(idx, i1)


def test_ballquery_module_and_local_ppf(dev):
    from PVCNN.modules import BallQuery
    import PVCNN.modules.functional as F
    xyz, nrm, _ = gaussian_clouds(2, 512, seed=8)
    xyz = xyz * np.float32(0.4)
    tx, tn = T(xyz, dev), T(nrm, dev)
    grouper = BallQuery(0.3, 128, include_coordinates=True)
    g = grouper(tx, tx, tn)  # [b, 6, u, n]
    # the model's local PPF block (pvcnn_classify.py:258-269) in torch
    d = tx.unsqueeze(2) - g[:, :3]
    dn = torch.norm(d, dim=1, p=2, keepdim=True)
    du = d / dn
    nr = g[:, 3:]
    cn = tn.unsqueeze(2).expand_as(nr)
    cos = torch.cat(((nr * du).sum(1, keepdim=True), (cn * du).sum(1, keepdim=True),
                     (nr * cn).sum(1, keepdim=True)), 1).clamp(-1, 1)
    idx = F.ball_query(tx, tx, 0.3, 128)
    lp = F.local_ppf(tx, tn, idx)  # fused kernel
    assert lp.shape == (2, 4, 128, 512)
    # compare in the cosine domain (acos is ill-conditioned near +-1) and |d|
    ok = torch.isfinite(cos).all(1)
    assert torch.allclose(torch.cos(lp[:, :3])[ok.unsqueeze(1).expand(-1, 3, -1, -1)],
                          cos[ok.unsqueeze(1).expand(-1, 3, -1, -1)], atol=2e-5)
    assert torch.allclose(lp[:, 3:], dn, atol=1e-5)


def test_pvconv_forward_backward(dev):
    from PVCNN.modules import PVConv
    torch.manual_seed(0)
    for shape in ("spherical", "cube"):
        m = PVConv(16, 32, "dgcnn_kernel", shape, 3, 8, with_coeff=True, with_se=True,
                   normalize=False).to(dev)
        xyz, _, feat = gaussian_clouds(2, 256, seed=3, c=16)
        tf = T(feat, dev).requires_grad_(True)
        out, _ = m((tf, T(xyz, dev)))
        assert out.shape == (2, 32, 256)
        out.sum().backward()
        assert torch.isfinite(tf.grad).all()
