"""CPU check of tests/golden/masked.npz (the reference's policy heads on fixed
logits, gen_golden.py): the recorded outputs agree with a float64 numpy
restatement of the masked categorical the GPU kernel implements, so the
GPU test (test_gpu_masked.py::test_masked_matches_reference_policy_heads)
pins the kernel to the reference's behaviour, not to a re-derivation."""
import os

import numpy as np
import pytest


@pytest.mark.parametrize("n", [6, 8])
def test_reference_policy_head_fixtures_are_the_masked_categorical(golden_dir, n):
    d = np.load(os.path.join(golden_dir, "masked.npz"))
    k = "N%d_" % n
    L = d[k + "logits"].astype(np.float64)
    nl = d[k + "nlegal"]
    R, nn = L.shape
    words = d[k + "legal"]
    legal = np.zeros((R, nn), bool)
    for a in range(nn):
        legal[:, a] = (words[:, a // 64] >> np.uint64(a % 64)) & np.uint64(1)
    assert np.array_equal(legal.sum(1), nl)
    x = np.where(legal, L, -np.inf)
    m = np.where(nl > 0, x.max(1), 0.0)
    lse = m + np.log(np.where(nl > 0, np.exp(x - m[:, None]).sum(1), 1.0))
    rows = np.arange(R)

    def lp(a):
        ok = (nl > 0) & (a >= 0) & (a < nn)
        ok[ok] &= legal[rows[ok], a[ok]]
        return np.where(ok, L[rows, np.clip(a, 0, nn - 1)] - lse, 0.0)

    live = nl > 0
    assert np.array_equal(d[k + "mode_action"][live], np.argmax(x, 1)[live])  # first max
    assert (d[k + "mode_action"][~live] == 0).all()  # model.py:69-71
    for key in ("mode", "sample", "eval"):
        np.testing.assert_allclose(d[k + key + "_logp"], lp(d[k + key + "_action"]), atol=2e-6)
    assert legal[rows[live], d[k + "sample_action"][live]].all()
    mm = L.max(1)
    p = np.exp(L - mm[:, None])
    ent = np.log(p.sum(1)) + mm - (p * L).sum(1) / p.sum(1)
    np.testing.assert_allclose(d[k + "full_entropy"], ent, atol=2e-6)
    pp = d[k + "ppo_probs"]
    np.testing.assert_allclose(pp[live], np.where(legal, np.exp(x - lse[:, None]), 0.0)[live], atol=2e-6)
    for i in np.flatnonzero(live):  # np.random.choice: searchsorted(cdf / cdf[-1], u, 'right')
        cdf = np.cumsum(pp[i])
        assert np.argmax(cdf / cdf[-1] > d[k + "ppo_u"][i]) == d[k + "ppo_action"][i]
