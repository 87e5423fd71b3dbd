"""Torch fp32 restatement of PVCNN_classifier.forward
(reference: PVCNN/models/pvcnn_classify.py:94-345, PVCNN/modules/pvconv.py:44-99)
for the model parity tests.

Every float operation of the hot path is plain differentiable torch here:
the local PPF math (:263-269), the voxel scatter-mean (index_add), the
devoxelisation (gather of the 8 corners, weighted sum), the dgcnn centre
gather.  The integer decisions -- ball-query neighbour lists, voxel indices
and counts, devox corner indices and weights -- come from the CPU oracle
(oracle/pcr_oracle.c, the parity anchor), evaluated on the same float
inputs the model's torch code produces.  The non-hot-path layers (Conv3d,
BatchNorm, SharedMLP, SE, classifier) are the model's own modules, so the
two forwards share weights and batch statistics.
"""
import numpy as np
import torch

import oracle


def _np(t):
    return t.detach().cpu().numpy()


def change_coords_torch(coords):
    """pvcnn_classify.py:154-184, the per-cloud Python loop."""
    b, _, n = coords.shape
    nc = coords - coords.mean(dim=2, keepdim=True)
    rank = torch.argsort(nc.norm(dim=1), dim=1, descending=True)
    bx = torch.zeros(b, 3, 1).to(nc)
    by = torch.zeros(b, 3, 1).to(nc)
    for i in range(b):
        x = nc[i, :, rank[i, 0]]
        x = x / x.norm()
        for j in range(1, n):
            y = nc[i, :, rank[i, j]]
            if y.norm() < 1e-5:
                continue
            y = y / y.norm()
            lam = (x * y).sum()
            if -0.9 < lam < 0.9:
                break
        bx[i, :, 0] = x
        by[i, :, 0] = y
    bx = bx - by * (bx.permute(0, 2, 1).bmm(by))
    bx = bx / bx.norm(dim=1, keepdim=True)
    bz = torch.cross(bx, by, dim=1)
    bz = bz / bz.norm(dim=1, keepdim=True)
    return torch.cat((bx.permute(0, 2, 1).bmm(nc), by.permute(0, 2, 1).bmm(nc),
                      bz.permute(0, 2, 1).bmm(nc)), dim=1)


def local_ppf_torch(coords, normals, radius, u):
    """:258-269 with the ball query (ball_query.cu:30-49) from the oracle."""
    idx = torch.from_numpy(oracle.ball_query(_np(coords), _np(coords), radius, u)).to(
        coords.device).long()                                   # [b, m, u]
    b, _, n = coords.shape
    flat = idx.reshape(b, 1, -1)
    gc = coords.gather(2, flat.expand(-1, 3, -1)).view(b, 3, n, u).permute(0, 1, 3, 2)
    gn = normals.gather(2, flat.expand(-1, 3, -1)).view(b, 3, n, u).permute(0, 1, 3, 2)
    nbr = gc - coords.unsqueeze(2)                              # grouper: p - c
    cc = coords.unsqueeze(2).expand(-1, -1, u, -1)
    cn = normals.unsqueeze(2).expand(-1, -1, u, -1)
    d = cc - nbr
    dn = torch.norm(d, dim=1, p=2, keepdim=True)
    du = d / dn
    nr_d = torch.acos(gn.mul(du).sum(dim=1, keepdim=True).clamp(-1, 1))
    ni_d = torch.acos(cn.mul(du).sum(dim=1, keepdim=True).clamp(-1, 1))
    nr_ni = torch.acos(gn.mul(cn).sum(dim=1, keepdim=True).clamp(-1, 1))
    return torch.cat((nr_d, ni_d, nr_ni, dn), dim=1)


def _scatter_mean(features, ind, cnt, r3):
    """Voxel means [b, c, r3] of the points with ind >= 0 (differentiable)."""
    b, c, n = features.shape
    out = features.new_zeros((b, c, r3))
    for i in range(b):
        ok = ind[i] >= 0
        out[i] = out[i].index_add(1, ind[i][ok], features[i][:, ok])
    return out / cnt.clamp(min=1).unsqueeze(1).to(features.dtype)


def _devox(grid, inds, wgts):
    """sum_q w_q grid[:, inds_q] per point; -1 rows contribute 0."""
    b, c, _ = grid.shape
    n = inds.shape[2]
    safe = inds.clamp(min=0)
    g = grid.gather(2, safe.reshape(b, 1, 8 * n).expand(-1, c, -1)).view(b, c, 8, n)
    w = torch.where(inds >= 0, wgts, torch.zeros_like(wgts))
    return (g * w.unsqueeze(1)).sum(dim=2)


def pvconv_torch(layer, features, coords):
    """PVConv.forward (pvconv.py:44-99) with torch float math."""
    b, c, n = features.shape
    r = layer.resolution
    r3 = r ** 3
    dev = features.device
    coords = coords.detach()
    centred = coords - coords.mean(2, keepdim=True)
    if layer.voxel_shape == "spherical":
        rad = centred.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values
        nc = centred / (rad + 1e-20)
        zero = np.zeros((b, 1, n), np.float32)
        _, ind, cnt = oracle.spherical_avg_voxelize_forward(zero, _np(nc), r)
        _, inds, wgts = oracle.spherical_trilinear_devoxelize_forward(
            r, _np(nc), np.zeros((b, 1, r3), np.float32), ind)
    else:
        vc = layer.voxelization
        if vc.normalize:
            scale = centred.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values
            nc = centred / (scale * 2.0 + vc.eps) + 0.5
        else:
            nc = (centred + 1) / 2.0
        nc = torch.clamp(nc * r, 0, r - 1)
        vox = torch.round(nc).to(torch.int32)
        zero = np.zeros((b, 1, n), np.float32)
        _, ind, cnt = oracle.avg_voxelize_forward(zero, _np(vox), r)
        _, inds, wgts = oracle.trilinear_devoxelize_forward(r, _np(nc),
                                                            np.zeros((b, 1, r3), np.float32))
    ind_t = torch.from_numpy(ind).to(dev).long()
    cnt_t = torch.from_numpy(cnt).to(dev)
    inds_t = torch.from_numpy(inds).to(dev).long()
    wgts_t = torch.from_numpy(wgts).to(dev)
    avg = _scatter_mean(features, ind_t, cnt_t, r3)
    vox_f = layer.voxel_layers(avg.view(b, c, r, r, r))
    vox_pt = _devox(vox_f.reshape(b, vox_f.shape[1], r3), inds_t, wgts_t)
    if layer.point_kernel_formal == "dgcnn_kernel":
        valid = (ind_t >= 0)
        center = avg.gather(2, ind_t.clamp(min=0).unsqueeze(1).expand(-1, c, -1))
        related = torch.where(valid.unsqueeze(1), features - center,
                              torch.zeros_like(features))
        point = layer.point_layers(torch.cat((related, features), 1))
    else:
        point = layer.point_layers(features)
    return (layer.coefficient * vox_pt + point) if layer.with_coeff else vox_pt + point


def classifier_forward_torch(model, inputs, local_ppf_from_oracle=True):
    """PVCNN_classifier.forward for the sph-dg / cu-dg configurations
    (change_coords or ppf preprocess, local PPF features)."""
    b, _, n = inputs.shape
    coords = inputs[:, :3, :]
    coords = coords - coords.mean(dim=2, keepdim=True)
    pre = model.rot_invariant_preprocess
    if pre == "change_coords":
        new = change_coords_torch(coords)
        features = new
        if model.extra_feature_channels == 4:
            # :200-209: global PPF against the mean point / raw mean normal
            normals = inputs[:, 3:6, :]
            cc = coords.mean(dim=2, keepdim=True).expand(-1, -1, n).contiguous()
            cn = normals.mean(dim=2, keepdim=True).expand(-1, -1, n).contiguous()
            ppfs = torch.from_numpy(oracle.spherical_ppf_forward(
                _np(coords), _np(cc), _np(normals.contiguous()), _np(cn))).to(inputs.device)
            features = torch.cat((features, ppfs), dim=1)
        if model.use_new_coords_for_voxel:
            coords = new
    elif pre == "ppf":
        normals = inputs[:, 3:6, :]
        normals = normals / normals.norm(dim=1, keepdim=True)
        cc = coords.mean(dim=2, keepdim=True).expand(-1, -1, n).contiguous()
        cn = normals.mean(dim=2, keepdim=True).expand(-1, -1, n).contiguous()
        features = torch.from_numpy(oracle.spherical_ppf_forward(
            _np(coords), _np(cc), _np(normals), _np(cn))).to(inputs.device)
    else:
        features = inputs
    if model.with_local_feat == "ppf":
        if local_ppf_from_oracle:
            # the oracle's local PPF (bit-exact with the kernel): the fuser's
            # max over the u neighbours routes each gradient to one argmax,
            # and a 1-ulp difference between two near-tied neighbours moves
            # it; torch's own local-PPF arithmetic is compared with the kernel
            # elementwise in test_local_ppf_fused_equals_composition
            nrm = inputs[:, 3:6, :].contiguous()
            cf = coords.contiguous()
            idx = oracle.ball_query(_np(cf), _np(cf), model.radius, model.neighbor_num)
            lp = torch.from_numpy(oracle.local_ppf(_np(cf), _np(nrm), _np(cf), _np(nrm), idx,
                                                   kmajor=False, relative=True)).to(inputs.device)
        else:
            lp = local_ppf_torch(coords, inputs[:, 3:6, :], model.radius, model.neighbor_num)
        features = torch.cat((features, model.fuser(lp).max(dim=2).values), dim=1)
    for layer in model.point_features:
        if hasattr(layer, "voxel_layers"):
            features = pvconv_torch(layer, features, coords)
        else:
            features = layer(features)
    if model.is_classify:
        return model.classifier(features.max(dim=2).values)
    return features
