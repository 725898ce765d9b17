"""GPU regression pins for hazards found in review:

* a live board loaded with an empty possible_moves (the reference can hold
  `possible_moves == []` on a non-terminated env before a reset,
  /root/reference/othello.py:242, and step() then takes the invalid path,
  :417-427) must take the invalid path in every kernel, including the fast
  k_play_rand / k_play_rand_w loops whose pick assumes a non-empty mask;
* the one position that exposed the gfx950 backend miscompile of the greedy
  bit planes on dword pairs ("A compiler hazard") must give
  GreedyPolicy's move (simple_policies.py:69-92) in every greedy kernel.
"""
import numpy as np
import pytest

from oracle import oracle

from test_gpu_parity import flags_of, get_state_np, make_env, t64, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


def _load_live_empty(torch, env, n, stride):
    """Mid-game state with every `stride`-th board's legal mask zeroed (still live)."""
    b, m, lg = get_state_np(env)
    lg = lg.copy()
    lg[::stride] = 0
    m = m.copy()
    m[::stride] &= ~np.uint16(2)  # live
    env.set_state(t64(torch, b), torch.from_numpy(m.view(np.int16)).cuda(), t64(torch, lg))
    return b, m, lg


@pytest.mark.parametrize("n", [6, 8, 10])
@pytest.mark.parametrize("policy", ["random", "greedy"])
def test_live_boards_without_moves_take_the_invalid_path(torch_cuda, n, policy):
    """step_policy with auto-reset and every output recorded (the fast kernels'
    configuration) on waves holding live boards whose possible_moves is empty:
    action -1, the invalid path (sudden death here), no overlapping colours;
    every action, reward, done, the final state and W/D/L equal the oracle."""
    torch = torch_cuda
    E, plies, stride = 4096, 40, 300
    env = make_env(torch, E, n, auto=True, seed=17)
    env.step_policy("random", n_plies=9)
    b, m, lg = _load_live_empty(torch, env, n, stride)
    env.counts(reset=True)
    acts, rews, dones = env.step_policy(policy, n_plies=plies)
    s = oracle.State(n, E)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    pid = 0 if policy == "random" else 1
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, False, True), pid, plies, seed=17, ply0=9)
    acts = acts.cpu().numpy()
    np.testing.assert_array_equal(acts, oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    b2, m2, lg2 = get_state_np(env)
    np.testing.assert_array_equal(b2, s.boards)
    np.testing.assert_array_equal(m2, s.meta)
    np.testing.assert_array_equal(lg2, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)
    assert (acts[0, ::stride] == -1).all() and (dones.cpu().numpy()[0, ::stride] == 1).all()
    W = oracle.nwords(n)
    assert not (b2[:, :W] & b2[:, W:]).any()


@pytest.mark.parametrize("n", [6, 8, 10])
def test_live_boards_without_moves_single_plies(torch_cuda, n):
    """The same through one-ply launches (the single-ply kernels) and through
    external steps with every action on such boards."""
    torch = torch_cuda
    E, stride = 2048, 300
    env = make_env(torch, E, n, auto=True, seed=19)
    env.step_policy("random", n_plies=7)
    b, m, lg = _load_live_empty(torch, env, n, stride)
    s = oracle.State(n, E)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    a1, r1, d1 = env.step_policy("random", n_plies=1)
    oa, orw, od, _ = oracle.rollout(s, flags_of(True, False, True), 0, 1, seed=19, ply0=7)
    np.testing.assert_array_equal(a1.cpu().numpy(), oa)
    np.testing.assert_array_equal(r1.cpu().numpy(), orw)
    np.testing.assert_array_equal(d1.cpu().numpy(), od)
    assert (a1.cpu().numpy()[0, ::stride] == -1).all()
    # external actions: any square is invalid on a board without moves
    b, m, lg = _load_live_empty(torch, env, n, stride)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    acts = np.random.RandomState(n).randint(-1, n * n + 1, size=E).astype(np.int32)
    for sd in (True, False):
        env2 = make_env(torch, E, n, sd=sd, auto=True, seed=19)
        env2.set_state(t64(torch, b), torch.from_numpy(m.view(np.int16)).cuda(), t64(torch, lg))
        s2 = oracle.State(n, E)
        s2.boards[:], s2.meta[:], s2.legal[:] = b, m, lg
        orw, od, _ = oracle.step(s2, flags_of(sd, False, True), acts, seed=19, ply=0)
        _, rew, dn, _ = env2.step(torch.from_numpy(acts).cuda(), observe=False)
        np.testing.assert_array_equal(rew.cpu().numpy(), orw)
        np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
        b2, m2, lg2 = get_state_np(env2)
        np.testing.assert_array_equal(b2, s2.boards)
        np.testing.assert_array_equal(m2, s2.meta)
        np.testing.assert_array_equal(lg2, s2.legal)


@pytest.mark.parametrize("n", [6, 8, 10])
def test_sample_step_on_live_boards_without_moves(torch_cuda, n):
    """oth_sample_step on live boards with no possible move: Policy.act's
    action 0 (model.py:69-71) and the invalid path, equal to the oracle's step."""
    torch = torch_cuda
    E, stride = 4096, 300
    env = make_env(torch, E, n, auto=True, seed=23)
    env.step_policy("random", n_plies=11)
    b, m, lg = _load_live_empty(torch, env, n, stride)
    logits = torch.randn(E, n * n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(n))
    acts, _, _, rew, dn = env.sample_step(logits, log_probs=False, entropy=False)
    a = acts.cpu().numpy()
    assert (a[::stride] == 0).all()
    s = oracle.State(n, E)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    orw, od, _ = oracle.step(s, flags_of(True, False, True), a, seed=23, ply=11)
    np.testing.assert_array_equal(rew.cpu().numpy(), orw)
    np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
    b2, m2, lg2 = get_state_np(env)
    np.testing.assert_array_equal(b2, s.boards)
    np.testing.assert_array_equal(m2, s.meta)
    np.testing.assert_array_equal(lg2, s.legal)


# The position of DESIGN.md's compiler hazard: white to move; GreedyPolicy
# (simple_policies.py:69-92) plays 31 (4 flips); the dword-pair planes inside
# k_play returned 33 (2 flips).
U2_BLACK, U2_WHITE, U2_LEGAL, U2_MOVE = 0x000020107b020409, 0x00001008040c0202, 0x0040402380310904, 31


def test_u2_miscompile_position_pinned(torch_cuda):
    torch = torch_cuda
    s = oracle.State(8, 1)
    s.boards[0] = [U2_BLACK, U2_WHITE]
    s.meta[0] = 1
    s.legal[0] = U2_LEGAL
    assert oracle.greedy(s)[0] == U2_MOVE  # the oracle simulates every move, as the reference
    for E in (1, 64, 300):
        boards = np.tile(np.array([[U2_BLACK, U2_WHITE]], dtype=np.uint64), (E, 1))
        meta = np.ones(E, dtype=np.uint16)
        legal = np.full((E, 1), U2_LEGAL, dtype=np.uint64)

        def fresh(auto):
            env = make_env(torch, E, 8, auto=auto)
            env.set_state(t64(torch, boards), torch.from_numpy(meta.view(np.int16)).cuda(), t64(torch, legal))
            return env
        # oth_policy_actions (k_policy_actions)
        assert (fresh(False).policy_actions("greedy").cpu().numpy() == U2_MOVE).all()
        # k_play<8, GREEDY, Fills> (no auto-reset: the generic ply loop), one ply
        a, _, _ = fresh(False).step_policy("greedy", n_plies=1)
        assert (a.cpu().numpy() == U2_MOVE).all()
        # k_play_rand<8, GREEDY> (auto-reset, every output recorded), one and two plies
        for plies in (1, 2):
            a, _, _ = fresh(True).step_policy("greedy", n_plies=plies)
            assert (a.cpu().numpy()[0] == U2_MOVE).all()
        # MaxiMinPolicy(1) is GreedyPolicy's argmax (simple_policies.py:111-155)
        assert (fresh(False).policy_actions("maximin1").cpu().numpy() == U2_MOVE).all()
