"""HIP-graph capture of the device RL loop: masked sampling + step enqueued by
the C ABI on torch's current stream, captured with torch.cuda.graph and
replayed, must equal the same plies run eagerly (state, actions, rewards,
dones, W/D/L) -- the launch-bound single-ply path of ppo.py-style training
 without per-ply host work.

Plain capture needs caller-supplied uniforms and initial_rand_steps = 0 (the
Philox counters are host values frozen at capture); VecOthelloEnv.graph_region
lifts that by advancing device offsets of both counters once per replay."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _ply(env, logits, u, rew, don, acts_out):
    act, _, _ = env.sample_actions(logits, uniforms=u, log_probs=False, entropy=False)
    env.step(act, rewards=rew, dones=don, observe=False)
    acts_out.copy_(act)


@pytest.mark.parametrize("n", [6, 8, 10])
def test_graph_replay_equals_eager(torch_gpu, n):
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    E, K = 3000, 16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    u = torch.rand(K, E, device=dev, generator=g)
    eager = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=9, device=dev)
    graphed = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=9, device=dev)
    eager.reset()
    graphed.reset()
    rew_e, don_e = torch.empty(K, E, dtype=torch.int32, device=dev), torch.empty(K, E, dtype=torch.uint8, device=dev)
    rew_g, don_g = torch.empty_like(rew_e), torch.empty_like(don_e)
    acts_e = torch.empty(K, E, dtype=torch.int32, device=dev)
    acts_g = torch.empty_like(acts_e)

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):  # records only: nothing runs during capture
        for k in range(K):
            _ply(graphed, logits, u[k], rew_g[k], don_g[k], acts_g[k])
    torch.cuda.synchronize()
    for _ in range(3):  # replays chain: the boards stay in HBM between them
        for k in range(K):
            _ply(eager, logits, u[k], rew_e[k], don_e[k], acts_e[k])
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(acts_g, acts_e)
        assert torch.equal(rew_g, rew_e)
        assert torch.equal(don_g, don_e)
        for x, y in zip(graphed.get_state(), eager.get_state()):
            assert torch.equal(x, y)
    assert np.array_equal(graphed.counts().cpu().numpy(), eager.counts().cpu().numpy())
    assert int(eager.counts().sum()) > 0


@pytest.mark.parametrize("n", [6, 8])
def test_graph_region_fresh_draws(torch_gpu, n):
    """graph_region: device-drawn samples (no uniforms) and random openings
    (initial_rand_steps > 0) under replay advance the Philox counters on the
    device, so replay r equals eager plies r*K .. r*K+K-1 of a twin env and two
    replays draw different actions."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    E, K = 2048, 8
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(100 + n)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    kw = dict(board_size=n, auto_reset=True, initial_rand_steps=4, seed=5, device=dev)
    eager, graphed = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    eager.reset()
    graphed.reset()
    acts_e = torch.empty(K, E, dtype=torch.int32, device=dev)
    acts_g = torch.empty_like(acts_e)

    def ply(env, k, out):
        act, _, _ = env.sample_actions(logits, log_probs=False, entropy=False)
        env.step(act, observe=False)
        out[k].copy_(act)

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph), graphed.graph_region():
        for k in range(K):
            ply(graphed, k, acts_g)
    torch.cuda.synchronize()
    prev = None
    for _ in range(3):
        with eager.graph_region():  # outside a capture: enqueues nothing
            for k in range(K):
                ply(eager, k, acts_e)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(acts_g, acts_e)
        for x, y in zip(graphed.get_state(), eager.get_state()):
            assert torch.equal(x, y)
        if prev is not None:
            assert not torch.equal(prev, acts_g)  # fresh draws per replay
        prev = acts_g.clone()
    # the device offsets hold what the replays consumed
    assert graphed.counter_offsets() == (3 * K, 3 * K)
    assert eager.counter_offsets() == (0, 0)
    assert np.array_equal(graphed.counts().cpu().numpy(), eager.counts().cpu().numpy())


def test_graph_region_step_vs_random_opponent(torch_gpu):
    """OthelloEnv-style plies (protagonist action + device random opponent,
    othello.py:176-200) captured inside graph_region: each replay's opponent
    draws equal an eager twin's."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    E, K, n = 2048, 6, 6
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    kw = dict(board_size=n, auto_reset=True, initial_rand_steps=2, seed=11, device=dev)
    eager, graphed = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    eager.reset_vs("random")
    graphed.reset_vs("random")
    out_e = torch.empty(K, 3, E, dtype=torch.int32, device=dev)
    out_g = torch.empty_like(out_e)

    def ply(env, k, out):
        act, _, _ = env.sample_actions(logits, log_probs=False, entropy=False)
        _, r, d, p = env.step_vs(act, opponent="random", observe=False)
        out[k, 0].copy_(r)
        out[k, 1].copy_(d)
        out[k, 2].copy_(p)

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph), graphed.graph_region():
        for k in range(K):
            ply(graphed, k, out_g)
    torch.cuda.synchronize()
    for _ in range(4):  # 24 calls, about 48 plies: 6x6 games end and auto-reset
        for k in range(K):
            ply(eager, k, out_e)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out_g, out_e)
        for x, y in zip(graphed.get_state(), eager.get_state()):
            assert torch.equal(x, y)
    assert int(out_e[:, 1].sum()) > 0  # games ended in the last replay (auto-reset with random openings)
