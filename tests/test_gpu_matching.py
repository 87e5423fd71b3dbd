"""GPU parity of the MFMA mutual-NN matching (SURVEY.md 8f row f1,
datasets/deepgmr_mn40.py:232-244) against the oracle: bit-exact -- both sum
the channels as k-ordered fmaf chains (include/pcr_math.h pcr_match_*)."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p,n1,n2,c", [(2, 300, 280, 64), (1, 257, 513, 33), (3, 1024, 1024, 64),
                                       (1, 128, 128, 512), (1, 1, 5, 3)])
def test_mutual_nn_matches_oracle(dev, p, n1, n2, c):
    from pcr_amd import ops
    rng = np.random.default_rng(p * 7 + n1 + c)
    f1 = rng.standard_normal((p, n1, c), dtype=np.float32)
    f2 = rng.standard_normal((p, n2, c), dtype=np.float32)
    got = ops.mutual_nn_match(torch.from_numpy(f1).to(dev), torch.from_numpy(f2).to(dev))
    torch.cuda.synchronize()
    exp = oracle.mutual_nn(f1, f2)
    for g, e, name in zip(got, exp, ("corr12", "corr21", "idx1", "idx2", "count")):
        assert np.array_equal(g.cpu().numpy(), e), name


def test_mutual_nn_permutation_and_ties(dev):
    from pcr_amd import ops
    rng = np.random.default_rng(5)
    n, c = 700, 32
    f1 = rng.standard_normal((n, c), dtype=np.float32)
    perm = rng.permutation(n)
    t1 = torch.from_numpy(f1).to(dev)
    t2 = torch.from_numpy(np.ascontiguousarray(f1[perm])).to(dev)
    idx1, idx2 = ops.find_correspondence_one_pair(t1, t2)
    assert torch.equal(idx1.cpu(), torch.arange(n))
    assert np.array_equal(idx2.cpu().numpy(), np.argsort(perm))
    # duplicated rows tie: the lowest index wins, as np.argmin
    f2 = np.concatenate([f1, f1], axis=0)
    got = ops.mutual_nn_match(t1.unsqueeze(0), torch.from_numpy(f2).to(dev).unsqueeze(0))
    exp = oracle.mutual_nn(f1[None], f2[None])
    for g, e in zip(got, exp):
        assert np.array_equal(g.cpu().numpy(), e)


@pytest.mark.parametrize("p,n1,n2,c", [(2, 300, 280, 64), (3, 1024, 1024, 64), (1, 257, 129, 33)])
def test_mutual_nn_channel_major(dev, p, n1, n2, c):
    """pcr_mutual_nn_match_cm on [p, c, n] features == the oracle on the
    transposes (same fmaf chains: bit-exact)."""
    from pcr_amd import ops
    rng = np.random.default_rng(p + n1 + 3 * c)
    f1 = rng.standard_normal((p, c, n1), dtype=np.float32)
    f2 = rng.standard_normal((p, c, n2), dtype=np.float32)
    got = ops.mutual_nn_match(torch.from_numpy(f1).to(dev), torch.from_numpy(f2).to(dev),
                              channel_major=True)
    exp = oracle.mutual_nn(np.ascontiguousarray(f1.transpose(0, 2, 1)),
                           np.ascontiguousarray(f2.transpose(0, 2, 1)))
    for g, e, name in zip(got, exp, ("corr12", "corr21", "idx1", "idx2", "count")):
        assert np.array_equal(g.cpu().numpy(), e), name
