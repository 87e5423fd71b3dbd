"""GPU parity of the fused extractor step (bench.py's workload) and of the
shared bit-exact math, plus full-size property tests."""
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


def expected_step(xyz, nrm, feat, k, r):
    """Composition of oracle ops = what one extractor step must produce."""
    ki_d, ki = oracle.knn_dir(xyz, xyz, k)
    lppf = oracle.local_ppf(xyz, nrm, xyz, nrm, ki, kmajor=True, relative=True)
    nc = oracle.normalize_sph(xyz)
    grid, ind, cnt = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    devox, dinds, dwgts = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    desc = devox.max(axis=2)
    return dict(knn_idx=ki, local_ppf=lppf, norm_coords=nc, ind=ind, cnt=cnt, grid=grid,
                devox=devox, dinds=dinds, dwgts=dwgts, desc=desc)


@pytest.mark.parametrize("b,n,c,k,r", [(1, 1024, 64, 16, 16), (4, 1024, 64, 32, 32),
                                       (2, 2048, 32, 32, 32), (2, 500, 7, 8, 9)])
def test_extractor_matches_oracle(dev, b, n, c, k, r):
    from pcr_amd.extractor import SphExtractor
    xyz, nrm, feat = gaussian_clouds(b, n, seed=n + b, c=c)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    out = ex.forward(T(xyz, dev), T(nrm, dev), T(feat, dev))
    torch.cuda.synchronize()
    exp = expected_step(xyz, nrm, feat, k, r)
    for key in ("knn_idx", "ind", "cnt", "dinds"):
        assert np.array_equal(N(out[key]), exp[key]), key
    for key in ("norm_coords", "grid", "dwgts", "devox", "desc"):
        assert np.array_equal(N(out[key]), exp[key]), key
    assert np.array_equal(N(out["local_ppf"]), exp["local_ppf"], equal_nan=True)


def test_extractor_graph_replay(dev):
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 8, 1024, 64, 32, 32
    xyz, nrm, feat = gaussian_clouds(b, n, seed=1, c=c)
    tx, tn, tf = T(xyz, dev), T(nrm, dev), T(feat, dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    ref = {kk: v.clone() for kk, v in ex.forward(tx, tn, tf).items()}
    ex.capture(tx, tn, tf)
    for _ in range(3):
        out = ex.replay()
    torch.cuda.synchronize()
    for key, v in ref.items():
        assert torch.equal(out[key], v) or torch.allclose(out[key], v, equal_nan=True), key


def poison(ex):
    """Every output and workspace buffer of the extractor set to all-ones
    bytes (NaN floats, -1 ints) before a run, so a checked result can only
    come from that run's kernels, never from an earlier call's leftovers."""
    import torch
    bufs = list(ex.outputs(0).values()) + list(ex.outputs(1).values())
    bufs += [ex.knn_ws, ex.ws] + list(ex._set(1))
    for t in bufs:
        t.view(-1).view(torch.uint8).fill_(0xFF)


def test_extractor_native_runner(dev):
    """pcr_extractor_run schedule 0 over the single buffer set (the native
    multi-step enqueue): every step's descriptor and the final outputs equal
    the single-step results; the removed schedules 1-5 are refused."""
    schedule = 0
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 8, 1024, 64, 32, 32
    xyz, nrm, feat = gaussian_clouds(b, n, seed=3, c=c)
    tx, tn, tf = T(xyz, dev), T(nrm, dev), T(feat, dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    ref = {kk: v.clone() for kk, v in ex.forward(tx, tn, tf).items()}
    # the runner's events are reused across calls of different lengths, with
    # and without grid-kernel timing (True: every step; an int N: the last N)
    for steps, timed in ((5, False), (3, True), (5, True), (6, 2), (1, False)):
        desc_steps = torch.empty((steps, b, c), device=dev)
        for _ in range(2):
            poison(ex)
            out = ex.run_native(tx, tn, tf, steps, desc_steps, schedule=schedule, timed=timed)
        torch.cuda.synchronize()
        for key, v in ref.items():
            if key == "desc":  # the runner writes each step's descriptor to desc_steps
                continue
            assert torch.equal(out[key], v) or torch.allclose(out[key], v, equal_nan=True), \
                (steps, key)
        for s in range(steps):
            assert torch.equal(desc_steps[s], ref["desc"]), (steps, s)
        if timed:
            ms = ex.grid_kernel_times()
            assert len(ms) == (0 if schedule == 0 else steps if timed is True else min(steps, timed))
            assert all(0 < t < 100 for t in ms)
    for gone in (1, 2, 3, 4, 5, 8):
        with pytest.raises(RuntimeError):
            ex.run_native(tx, tn, tf, 2, schedule=gone)


@pytest.mark.parametrize("schedule", [0, 6, 7])
def test_extractor_runner_batch_ring(dev, schedule):
    """pcr_extractor_run over a batch ring of 3 distinct batches (each with
    its own output set): one call of 3 steps, then a call of 5 steps that
    continues the cycle at set0 = 3 % 3 and wraps (sets 0 and 1 written
    twice, by batches 0 and 1 again).  After each call every set holds the
    oracle's outputs of its batch; desc_steps holds every step's
    descriptor."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 4, 1024, 16, 32, 32
    batches = [gaussian_clouds(b, n, seed=80 + i, c=c) for i in range(3)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches]
    exp = [expected_step(*bt, k, r) for bt in batches]
    ex = SphExtractor(b, n, c, k, r, device=dev)
    set0 = 0
    for steps in (3, 5):
        ring = ex.ring_outputs(3)
        for o in ring:
            for t in o.values():
                t.view(-1).view(torch.uint8).fill_(0xFF)
        desc_steps = torch.full((steps, b, c), float("nan"), device=dev)
        ex.run_ring(tb, steps, set0, desc_steps, schedule=schedule)
        torch.cuda.synchronize()
        for i in range(3):
            for key in ("knn_idx", "ind", "cnt", "dinds", "dwgts", "norm_coords", "grid",
                        "devox"):
                assert np.array_equal(N(ring[i][key]), exp[i][key]), (steps, i, key)
            assert np.array_equal(N(ring[i]["local_ppf"]), exp[i]["local_ppf"],
                                  equal_nan=True), (steps, i)
        for s in range(steps):
            assert np.array_equal(N(desc_steps[s]), exp[(set0 + s) % 3]["desc"]), (steps, s)
        set0 = (set0 + steps) % 3


def test_extractor_runner_ring_list_mutated(dev):
    """run_ring skips re-checking a call's batch tuples when they are the
    ones of the previous call; a tuple replaced in the SAME list object is
    checked and keyed again: its set then holds the new batch's outputs, and
    a replacement of the wrong shape is refused."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 4, 1024, 16, 32, 32
    batches = [gaussian_clouds(b, n, seed=140 + i, c=c) for i in range(4)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches[:3]]
    ex = SphExtractor(b, n, c, k, r, device=dev)
    ring = ex.ring_outputs(3)
    ex.run_ring(tb, 3, 0, schedule=6)
    ex.run_ring(tb, 3, 0, schedule=6)  # the cached path
    tb[1] = tuple(T(a, dev) for a in batches[3])
    ex.run_ring(tb, 3, 0, schedule=6)
    torch.cuda.synchronize()
    exp = expected_step(*batches[3], k, r)
    for key in ("knn_idx", "ind", "cnt", "grid", "devox"):
        assert np.array_equal(N(ring[1][key]), exp[key]), key
    tb[2] = (tb[2][0][:, :, :512].contiguous(), tb[2][1], tb[2][2])
    with pytest.raises(RuntimeError):
        ex.run_ring(tb, 3, 0, schedule=6)


@pytest.mark.parametrize("schedule,rings", [(6, ((2, 5), (5, 7))), (7, ((3, 7), (4, 9)))])
def test_extractor_runner_multi_queue_rings(dev, schedule, rings):
    """Schedules 6 (two voxel + two KNN queues) and 7 (three voxel + one
    KNN queue) over rings that one call wraps: a ring size that is a
    multiple of the voxel queue count rewrites each set on its own queue (no
    ring events: 2 sets x 5 steps, 3 x 7), another size on another queue
    behind the per-set event (5 x 7, 4 x 9).  The single-set runner refuses
    both, and a ring smaller than the voxel queue count is refused."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 4, 1024, 16, 32, 32
    batches = [gaussian_clouds(b, n, seed=110 + i, c=c) for i in range(5)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches]
    exp = [expected_step(*bt, k, r) for bt in batches]
    ex = SphExtractor(b, n, c, k, r, device=dev)
    for R, steps in rings:
        ring = ex.ring_outputs(R)
        for o in ring:
            for t in o.values():
                t.view(-1).view(torch.uint8).fill_(0xFF)
        desc_steps = torch.full((steps, b, c), float("nan"), device=dev)
        ex.run_ring(tb[:R], steps, 0, desc_steps, schedule=schedule)
        torch.cuda.synchronize()
        for i in range(R):
            for key in ("knn_idx", "ind", "cnt", "dinds", "dwgts", "norm_coords", "grid",
                        "devox"):
                assert np.array_equal(N(ring[i][key]), exp[i][key]), (R, i, key)
            assert np.array_equal(N(ring[i]["local_ppf"]), exp[i]["local_ppf"],
                                  equal_nan=True), (R, i)
        for s in range(steps):
            assert np.array_equal(N(desc_steps[s]), exp[s % R]["desc"]), (R, s)
    with pytest.raises(RuntimeError):
        ex.run_native(*tb[0], 2, schedule=schedule)
    with pytest.raises(RuntimeError):
        ex.run_ring(tb[:schedule - 5], 2, schedule=schedule)


@pytest.mark.parametrize("b,n,c,r", [(3, 1000, 7, 16), (2, 300, 5, 32), (4, 1024, 64, 32),
                                     (2, 1, 3, 16), (5, 64, 1, 16)])
@pytest.mark.parametrize("with_desc", [True, False])
def test_voxel_back_half_variants_identical(dev, b, n, c, r, with_desc):
    """The two back halves of the split voxel stage after one prep give the
    same bits: means_devox + stream (the reference composition) and means +
    stream_devox (devox + descriptor inside the grid stream, the c2 product
    path) -- grid, cnt, devox and desc (NULL desc included), at clouds below
    1024 points, odd channel counts (a last item with one channel) and a
    one-point cloud; one size also against the oracle."""
    from pcr_amd import _lib
    from pcr_amd.ops import _ptr
    lib = _lib.load()
    assert lib.pcr_extractor_stream_devox_ok(n, c, r)
    xyz, _, feat = gaussian_clouds(b, n, seed=7 * n + c, c=c)
    tx, tf = T(xyz, dev), T(feat, dev)
    r3 = r ** 3
    ws = torch.empty(lib.pcr_extractor_workspace_size(b, n, c, r), dtype=torch.uint8, device=dev)
    e = torch.empty
    nc, ind = e((b, 3, n), device=dev), e((b, n), dtype=torch.int32, device=dev)
    dinds, dwgts = e((b, 8, n), dtype=torch.int32, device=dev), e((b, 8, n), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.pcr_extractor_voxel_prep(_ptr(tx), b, n, r, _ptr(nc), _ptr(ind), _ptr(dinds),
                                            _ptr(dwgts), _ptr(ws), ws.numel(), st), "prep")
    outs = []
    for variant in range(2):
        cnt = torch.full((b, r3), -7, dtype=torch.int32, device=dev)
        grid = torch.full((b, c, r3), float("nan"), device=dev)
        devox = torch.full((b, c, n), float("nan"), device=dev)
        desc = torch.full((b, c), float("nan"), device=dev) if with_desc else None
        if variant == 0:
            # means_devox needs a descriptor buffer: a scratch one when desc is NULL
            d0 = desc if with_desc else e((b, c), device=dev)
            _lib.check(lib.pcr_extractor_voxel_means_devox(
                _ptr(tf), b, c, n, r, _ptr(devox), _ptr(dinds), _ptr(dwgts), _ptr(d0),
                _ptr(ws), ws.numel(), st), "means_devox")
            _lib.check(lib.pcr_extractor_voxel_stream(b, c, n, r, _ptr(cnt), _ptr(grid), _ptr(ws),
                                                      ws.numel(), st), "stream")
        elif variant == 1:
            _lib.check(lib.pcr_extractor_voxel_means(_ptr(tf), b, c, n, r, _ptr(ws), ws.numel(),
                                                     st), "means")
            _lib.check(lib.pcr_extractor_voxel_stream_devox(
                b, c, n, r, _ptr(cnt), _ptr(grid), _ptr(devox), _ptr(dwgts), _ptr(desc),
                _ptr(ws), ws.numel(), st), "stream_devox")
        outs.append((cnt, grid, devox, desc))
    torch.cuda.synchronize()
    for v in (1,):
        for name, a, o in zip(("cnt", "grid", "devox", "desc"), outs[0], outs[v]):
            if a is None:
                assert o is None
                continue
            assert torch.equal(a, o), (v, name)
    if b == 3:
        ref = expected_step(xyz, gaussian_clouds(b, n, seed=7 * n + c, c=c)[1], feat, 1, r)
        cnt, grid, devox, desc = outs[1]
        assert np.array_equal(N(cnt), ref["cnt"]) and np.array_equal(N(grid), ref["grid"])
        assert np.array_equal(N(devox), ref["devox"])
        if with_desc:
            assert np.array_equal(N(desc), ref["desc"])


def test_extractor_full_size_properties(dev):
    """BASELINE c2 shape: 32 x 1024, k=32, r=32, C=64 -- size-independent
    properties: ind consistent with cnt, grid empty where cnt == 0, the grid
    mean reproduces the per-voxel mean, knn slot 0 is at distance 0."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 32, 1024, 64, 32, 32
    xyz, nrm, feat = gaussian_clouds(b, n, seed=7, c=c)
    ex = SphExtractor(b, n, c, k, r, device=dev, with_dist=True)
    out = ex.forward(T(xyz, dev), T(nrm, dev), T(feat, dev))
    torch.cuda.synchronize()
    ind, cnt, grid = out["ind"].long(), out["cnt"], out["grid"]
    valid = ind >= 0
    hist = torch.zeros_like(cnt)
    for bi in range(b):
        hist[bi].index_add_(0, ind[bi][valid[bi]], torch.ones_like(ind[bi][valid[bi]],
                                                                   dtype=cnt.dtype))
    assert torch.equal(hist, cnt)
    empty = (cnt == 0).unsqueeze(1).expand_as(grid)
    assert (grid[empty] == 0).all()
    sums = torch.zeros_like(grid)
    tf = T(feat, dev)
    for bi in range(b):
        sums[bi].index_add_(1, ind[bi][valid[bi]], tf[bi][:, valid[bi]])
    mean = sums / cnt.clamp(min=1).unsqueeze(1)
    assert torch.allclose(mean, grid, atol=1e-5)
    assert (ex.knn_dist[:, 0, :] == 0).all()
    # full-size bit-exact check on two clouds against the oracle
    exp = expected_step(xyz[:2], nrm[:2], feat[:2], k, r)
    for key in ("knn_idx", "ind", "cnt", "grid", "devox"):
        assert np.array_equal(N(out[key][:2]), exp[key]), key


def test_device_math_bit_exact(dev):
    """pcr_math.h evaluated on gfx950 == the same code on the host."""
    import ctypes
    from pcr_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(0)
    n = 1 << 20
    x = np.concatenate([rng.uniform(-1, 1, n - 8),
                        [-1, 1, 0, -0.0, 0.5, -0.5, 1e-30, np.nextafter(1, 0)]]).astype(np.float32)
    tx = T(x, dev)
    out = torch.empty_like(tx)
    s = torch.cuda.current_stream().cuda_stream
    for op, ref in ((0, oracle.acosf), (1, oracle.atanf)):
        _lib.check(lib.pcr_selftest_math(op, tx.data_ptr(), None, n, 0, out.data_ptr(), None, s),
                   "selftest")
        assert np.array_equal(N(out), ref(x)), op
    t = (rng.standard_normal(n) * 10).astype(np.float32)
    tt = T(t, dev)
    _lib.check(lib.pcr_selftest_math(1, tt.data_ptr(), None, n, 0, out.data_ptr(), None, s), "st")
    assert np.array_equal(N(out), oracle.atanf(t))
    pos = np.abs(t).astype(np.float32)
    tp = T(pos, dev)
    _lib.check(lib.pcr_selftest_math(2, tp.data_ptr(), None, n, 0, out.data_ptr(), None, s), "st")
    assert np.array_equal(N(out), np.sqrt(pos))
    y = rng.standard_normal(n).astype(np.float32)
    ty = T(y, dev)
    _lib.check(lib.pcr_selftest_math(3, tt.data_ptr(), ty.data_ptr(), n, 0, out.data_ptr(), None,
                                     s), "st")
    assert np.array_equal(N(out), (t / y).astype(np.float32))
    # double sqrt / div / fma / acos
    xd = rng.uniform(0, 4, n)
    yd = rng.uniform(0.1, 4, n)
    txd, tyd = T(xd, dev), T(yd, dev)
    od = torch.empty_like(txd)
    _lib.check(lib.pcr_selftest_math_d(2, txd.data_ptr(), None, n, od.data_ptr(), s), "st")
    assert np.array_equal(N(od), np.sqrt(xd))
    _lib.check(lib.pcr_selftest_math_d(3, txd.data_ptr(), tyd.data_ptr(), n, od.data_ptr(), s),
               "st")
    assert np.array_equal(N(od), xd / yd)
    xa = rng.uniform(-1, 1, n)
    txa = T(xa, dev)
    _lib.check(lib.pcr_selftest_math_d(0, txa.data_ptr(), None, n, od.data_ptr(), s), "st")
    assert np.array_equal(N(od), oracle.acos_d(xa))
    # spherical voxel index over many points, r = 32
    xyz, _, _ = gaussian_clouds(1, 1 << 18, seed=3)
    nc = oracle.normalize_sph(xyz)[0]
    ti = torch.empty(nc.shape[1], dtype=torch.int32, device=dev)
    tnc = T(nc, dev)
    _lib.check(lib.pcr_selftest_math(4, tnc.data_ptr(), None, nc.shape[1], 32, None,
                                     ti.data_ptr(), s), "st")
    assert np.array_equal(N(ti), oracle.sph_index(nc, 32))
    del ctypes


@pytest.mark.parametrize("seed", [0, 1])
def test_extractor_ind_vs_reference_fp32_normalisation(dev, seed):
    """BASELINE c2 (32 x 1024, r = 32): the extractor's voxel indices (its
    fixed-order fp64 normalisation) against the spherical voxelisation of
    the coords the reference's Spherical_Voxelization.forward produces with
    torch fp32 on the GPU (PVCNN/modules/spherical_vox.py:17-19).  Every
    point in a different voxel must sit on a bin edge (tests/edges.py); the
    count is printed."""
    import edges
    from pcr_amd import ops
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r = 32, 1024, 64, 32, 32
    xyz, nrm, feat = gaussian_clouds(b, n, seed=seed, c=c)
    tx, tn, tf = T(xyz, dev), T(nrm, dev), T(feat, dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    out = ex.forward(tx, tn, tf)
    ind_ext, nc_ext = N(out["ind"]).copy(), N(out["norm_coords"]).copy()
    nc_ref = tx - tx.mean(2, keepdim=True)
    nc_ref = nc_ref / (nc_ref.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values + 1e-20)
    nc_ref = nc_ref.contiguous()
    _, ind_ref, _ = ops.spherical_avg_voxelize_forward(tf, nc_ref, r)
    torch.cuda.synchronize()
    ind_ref, nc_ref = N(ind_ref), N(nc_ref)
    assert np.abs(nc_ext - nc_ref).max() <= 1e-6
    total = 0
    for i in range(b):
        d, e, worst = edges.explain(nc_ext[i], nc_ref[i], ind_ext[i], ind_ref[i], r)
        total += d
        assert d == e, "cloud %d: %d indices differ, %d on a bin edge (worst %.3g)" % (i, d, e,
                                                                                      worst)
    print("c2 seed %d: %d of %d points in a different voxel than under the reference's "
          "torch-fp32 normalisation, all on bin edges" % (seed, total, b * n))
    assert total <= b * n // 1000


@pytest.mark.parametrize("prefetch", [False, True, "voxel_ahead"])
@pytest.mark.parametrize("b,n,c,k,r", [(4, 1024, 16, 32, 16), (2, 2048, 32, 32, 32),
                                       (3, 1500, 7, 16, 16)])
def test_extractor_pipelined_steps(dev, b, n, c, k, r, prefetch):
    """SphExtractor.pipelined_steps (bench.py c3: each batch's KNN + local
    PPF on s_nbr one batch ahead of the caller's voxel side and backwards;
    voxel_ahead: each batch's voxel head too, on s_vox, with alternating
    voxel output sets): every step sees exactly its own batch's outputs,
    equal to the oracle, and the consume callback's devox backward equals
    the serial one."""
    from pcr_amd import ops
    from pcr_amd.extractor import SphExtractor
    batches = [gaussian_clouds(b, n, seed=40 + s, c=c) for s in range(4)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches]
    gy = torch.randn((b, c, n), generator=torch.Generator().manual_seed(5)).to(dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    poison(ex)
    got = []

    def consume(s, out):
        gg = ops.spherical_trilinear_devoxelize_backward(gy, out["dinds"], out["dwgts"], r)
        got.append(({kk: v.clone() for kk, v in out.items()}, gg))

    ex.pipelined_steps(4, lambda s: tb[s], consume, prefetch=bool(prefetch),
                       voxel_ahead=prefetch == "voxel_ahead")
    torch.cuda.synchronize()
    assert len(got) == 4
    for s, (out, gg) in enumerate(got):
        exp = expected_step(*batches[s], k, r)
        for key in ("knn_idx", "ind", "cnt", "dinds", "grid", "devox", "desc"):
            assert np.array_equal(N(out[key]), exp[key]), (s, key)
        assert np.array_equal(N(out["local_ppf"]), exp["local_ppf"], equal_nan=True), s
        ref = ops.spherical_trilinear_devoxelize_backward(gy, T(exp["dinds"], dev),
                                                          T(exp["dwgts"], dev), r)
        assert torch.equal(gg, ref), s


def _check_steps(got, batches, k, r):
    assert len(got) == len(batches)
    for s, out in enumerate(got):
        exp = expected_step(*batches[s], k, r)
        for key in ("knn_idx", "ind", "cnt", "dinds", "grid", "devox", "desc"):
            assert np.array_equal(N(out[key]), exp[key]), (s, key)
        assert np.array_equal(N(out["local_ppf"]), exp["local_ppf"], equal_nan=True), s


def test_extractor_pipelined_batches_made_in_loop(dev):
    """pipelined_steps with batch(s) making its tensors on the caller's stream
    inside the loop, as train.py:140 does (inputs.to(device)): each batch is
    uploaded after a GPU-side delay on the current stream, into fresh
    buffers, and then scaled in place (x * 2 / 2, exact), so a neighbour
    stream that is not ordered after the producer reads unwritten memory.
    Every step against the oracle."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r, steps = 4, 1024, 16, 32, 32, 5
    batches = [gaussian_clouds(b, n, seed=60 + s, c=c) for s in range(steps)]
    staged = [[T(a * np.float32(2.0), dev) for a in bt] for bt in batches]
    ex = SphExtractor(b, n, c, k, r, device=dev)
    got = []

    def batch(s):
        torch.cuda._sleep(2_000_000)  # the producer lags behind the host
        out = []
        for src in staged[s]:
            t = torch.empty_like(src)
            t.copy_(src)  # device to device: asynchronous on the current stream
            t.div_(2.0)
            out.append(t)
        return tuple(out)

    ex.pipelined_steps(steps, batch, lambda s, out: got.append(
        {kk: v.clone() for kk, v in out.items()}))
    torch.cuda.synchronize()
    _check_steps(got, batches, k, r)


def test_extractor_pipelined_in_place_producer(dev):
    """The default pipelined_steps (prefetch=False) with a producer that
    refills ONE staging buffer in place each step (xyz.copy_(host), as a
    loader with a pinned staging tensor does), after a GPU-side delay: step
    s+1's copy must not overwrite step s's inputs while its voxel side or
    KNN still read them.  Every step against the oracle."""
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r, steps = 4, 1024, 16, 32, 32, 5
    batches = [gaussian_clouds(b, n, seed=80 + s, c=c) for s in range(steps)]
    src = [[T(a, dev) for a in bt] for bt in batches]
    stage = [torch.empty_like(t) for t in src[0]]
    ex = SphExtractor(b, n, c, k, r, device=dev)
    got = []

    def batch(s):
        torch.cuda._sleep(2_000_000)  # the producer lags behind the host
        for dst, t in zip(stage, src[s]):
            dst.copy_(t)
        return tuple(stage)

    ex.pipelined_steps(steps, batch, lambda s, out: got.append(
        {kk: v.clone() for kk, v in out.items()}))
    torch.cuda.synchronize()
    _check_steps(got, batches, k, r)


def test_extractor_pipelined_after_serial_forward(dev):
    """The sequence behind the round-3 illegal-address fault: a serial
    forward whose consume allocates and frees a large gradient on the
    caller's stream, then pipelined_steps on the same extractor (index set 1
    made on the first pipelined call, not pre-made by poison()).  Every
    pipelined step against the oracle."""
    from pcr_amd import ops
    from pcr_amd.extractor import SphExtractor
    b, n, c, k, r, steps = 8, 2048, 64, 32, 32, 4
    batches = [gaussian_clouds(b, n, seed=70 + s, c=c) for s in range(steps)]
    tb = [tuple(T(a, dev) for a in bt) for bt in batches]
    gy = torch.randn((b, c, n), generator=torch.Generator().manual_seed(6)).to(dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    out = ex.forward(*tb[0])
    gg = ops.spherical_trilinear_devoxelize_backward(gy, out["dinds"], out["dwgts"], r)
    gx = ops.spherical_avg_voxelize_backward(gg, out["ind"], out["cnt"])
    del gg, gx  # freed with their kernels possibly still pending
    got = []

    def consume(s, o):
        g2 = ops.spherical_trilinear_devoxelize_backward(gy, o["dinds"], o["dwgts"], r)
        ops.spherical_avg_voxelize_backward(g2, o["ind"], o["cnt"])
        got.append({kk: v.clone() for kk, v in o.items()})

    ex.pipelined_steps(steps, lambda s: tb[s], consume)
    torch.cuda.synchronize()
    _check_steps(got, batches, k, r)
