"""The play kernels' 4-ply groups at launch boundaries (round 6): greedy play
with random openings runs its plies in groups of four from a multiple of 4, with
a partial group at either end of a launch; multi-word random play has a loop
with the opening bookkeeping and one without.  Launches of odd lengths must give
the plies one launch gives, and the oracle's replay (device.hpp k_play_rand,
k_play_rand_w; the Philox draw of ply g is word g % 4 of block g / 4)."""
import numpy as np
import pytest

from oracle import oracle

from test_gpu_parity import flags_of, get_state_np, make_env, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

CHUNKS = (3, 7, 1, 2, 5, 10, 4, 6, 9, 13)  # 60 plies, every ply0 % 4 and launch length % 4


def _chunked(torch, env, policy):
    parts = [env.step_policy(policy, n_plies=k) for k in CHUNKS]
    return tuple(torch.cat([p[i] for p in parts]) for i in range(3))


@pytest.mark.parametrize("n,policy,init_rand,dr", [(8, "greedy", 10, False), (8, "greedy", 6, True),
                                                   (6, "greedy", 4, False), (10, "random", 6, True),
                                                   (10, "random", 0, True), (8, "random", 6, False)])
def test_odd_launches_equal_one_launch_and_oracle(torch_cuda, n, policy, init_rand, dr):
    torch = torch_cuda
    E, plies = 4096, sum(CHUNKS)
    one = make_env(torch, E, n, dr=dr, auto=True, seed=5, init_rand=init_rand)
    one.reset()
    a1, r1, d1 = one.step_policy(policy, n_plies=plies)
    many = make_env(torch, E, n, dr=dr, auto=True, seed=5, init_rand=init_rand)
    many.reset()
    a2, r2, d2 = _chunked(torch, many, policy)
    assert torch.equal(a1, a2) and torch.equal(r1, r2) and torch.equal(d1, d2)
    for x, y in zip(one.get_state(), many.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(one.counts(), many.counts())
    s = oracle.reset_openings(n, E, 5, 0, 0, init_rand) if init_rand else oracle.reset(n, E)
    pid = 0 if policy == "random" else 1
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, dr, True), pid, plies, seed=5,
                                       initial_rand_steps=init_rand)
    np.testing.assert_array_equal(a1.cpu().numpy(), oa)
    np.testing.assert_array_equal(r1.cpu().numpy(), orw)
    np.testing.assert_array_equal(d1.cpu().numpy(), od)
    b, m, lg = get_state_np(many)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(many.counts().cpu().numpy(), owdl)
