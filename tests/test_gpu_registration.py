"""One rank's registration-pair step (BASELINE c4; datasets/deepgmr_mn40.py:
71-97 extracts both clouds of a pair, :232-244 matches them) against the
oracle composition: extractor outputs of the 2P clouds bit-exact, and the
mutual-NN matching of each source's devoxelised features against its
target's equal to oracle.mutual_nn on the oracle's devox."""
import numpy as np
import pytest
import torch

import oracle
from clouds import gaussian_clouds

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def oracle_pair_step(xyz, nrm, feat, k, r, p):
    _, ki = oracle.knn_dir(xyz, xyz, k)
    nc = oracle.normalize_sph(xyz)
    grid, ind, cnt = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    devox, _, _ = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    f1 = np.ascontiguousarray(devox[:p].transpose(0, 2, 1))
    f2 = np.ascontiguousarray(devox[p:].transpose(0, 2, 1))
    return dict(knn_idx=ki, ind=ind, cnt=cnt, grid=grid, devox=devox, desc=devox.max(axis=2),
                match=oracle.mutual_nn(f1, f2))


@pytest.mark.parametrize("p,n,c,k,r", [(3, 1024, 32, 16, 16), (2, 1024, 64, 32, 32)])
def test_pair_step_matches_oracle(dev, p, n, c, k, r):
    from pcr_amd.registration import PairExtractor
    xyz, nrm, feat = gaussian_clouds(2 * p, n, seed=40 + p, c=c)
    # targets: the sources rotated and permuted, as a registration pair
    rng = np.random.default_rng(p)
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    for i in range(p):
        perm = rng.permutation(n)
        xyz[p + i] = (q @ xyz[i])[:, perm]
        nrm[p + i] = (q @ nrm[i])[:, perm]
        feat[p + i] = feat[i][:, perm]
    xyz, nrm = xyz.astype(np.float32), nrm.astype(np.float32)
    exp = oracle_pair_step(xyz, nrm, feat, k, r, p)
    pe = PairExtractor(p, n, c, k, r, device=dev)
    tx, tn, tf = T(xyz, dev), T(nrm, dev), T(feat, dev)
    out = pe.forward(tx, tn, tf)
    torch.cuda.synchronize()
    for key in ("knn_idx", "ind", "cnt", "grid", "devox", "desc"):
        assert np.array_equal(N(out[key]), exp[key]), key
    for g, e, name in zip((out[x] for x in ("corr12", "corr21", "idx1", "idx2", "count")),
                          exp["match"], ("corr12", "corr21", "idx1", "idx2", "count")):
        assert np.array_equal(N(g), e), name
    # the native runner's per-step matching gives the same, every step
    from test_gpu_extractor import poison
    for schedule in (0,):
        desc_steps = torch.empty((4, 2 * p, c), device=dev)
        poison(pe.ex)
        for t in (pe.match.corr12, pe.match.corr21, pe.match.idx1, pe.match.idx2,
                  pe.match.count):
            t.view(-1).view(torch.uint8).fill_(0xFF)
        nat = pe.run_native(tx, tn, tf, 4, desc_steps, schedule=schedule)
        torch.cuda.synchronize()
        for key in ("knn_idx", "ind", "cnt", "grid", "devox"):  # desc: desc_steps below
            assert np.array_equal(N(nat[key]), exp[key]), (schedule, key)
        for g, e, name in zip((nat[x] for x in ("corr12", "corr21", "idx1", "idx2", "count")),
                              exp["match"], ("corr12", "corr21", "idx1", "idx2", "count")):
            assert np.array_equal(N(g), e), (schedule, name)
        for s in range(4):
            assert np.array_equal(N(desc_steps[s]), exp["desc"]), (schedule, s)


def test_pair_runner_rejects_odd_batch(dev):
    from pcr_amd.extractor import SphExtractor
    from pcr_amd.registration import PairMatch
    ex = SphExtractor(3, 256, 8, 8, 8, device=dev)
    xyz, nrm, feat = gaussian_clouds(3, 256, seed=1, c=8)
    with pytest.raises(RuntimeError):
        ex.run_native(T(xyz, dev), T(nrm, dev), T(feat, dev), 1,
                      match=PairMatch(1, 256, dev))


def _pair_batch(p, n, c, seed):
    xyz, nrm, feat = gaussian_clouds(2 * p, n, seed=seed, c=c)
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    for i in range(p):
        perm = rng.permutation(n)
        xyz[p + i] = (q @ xyz[i])[:, perm]
        nrm[p + i] = (q @ nrm[i])[:, perm]
        feat[p + i] = feat[i][:, perm]
    return xyz.astype(np.float32), nrm.astype(np.float32), feat


@pytest.mark.parametrize("schedule", [0, 6, 7])
def test_pair_runner_batch_ring(dev, schedule):
    """BASELINE c4 over distinct pair batches (datasets/deepgmr_mn40.py:71-97,
    a new pair per item): the native runner's batch ring, 4 batches of 2
    pairs, two calls of 4 steps (schedule 6 matches consecutive steps on two
    queues at once, each in its own half of the matching workspace); after
    each call every ring set's extractor outputs and matching against the
    oracle of its batch."""
    from pcr_amd.registration import PairExtractor
    p, n, c, k, r = 2, 1024, 32, 32, 32
    batches = [_pair_batch(p, n, c, 90 + i) for i in range(4)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches]
    exp = [oracle_pair_step(*bt, k, r, p) for bt in batches]
    pe = PairExtractor(p, n, c, k, r, device=dev)
    for call in range(2):
        ring = pe.ex.ring_outputs(4, p)
        for o in ring:
            for t in o.values():
                t.view(-1).view(torch.uint8).fill_(0xFF)
        pe.run_ring(tb, 4, schedule=schedule)
        torch.cuda.synchronize()
        for i in range(4):
            for key in ("knn_idx", "ind", "cnt", "grid", "devox", "desc"):
                assert np.array_equal(N(ring[i][key]), exp[i][key]), (call, i, key)
            for name, e in zip(("corr12", "corr21", "idx1", "idx2", "count"), exp[i]["match"]):
                assert np.array_equal(N(ring[i][name]), e), (call, i, name)
