"""GPU parity: the HIP engine (through the C ABI) against the reference's golden
fixtures and the CPU oracle, bit for bit.  Run on an MI355X (`-m gpu`)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

SIZES = list(range(4, 17))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def t64(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def np_u64(t):
    return t.cpu().numpy().view(np.uint64)


def flags_of(sd, dr, auto=False):
    return ((oracle.F_SUDDEN_DEATH if sd else 0) | (oracle.F_DISK_REWARD if dr else 0) |
            (oracle.F_AUTO_RESET if auto else 0))


def make_env(torch, E, n, sd=True, dr=False, auto=False, seed=0, id_base=0, init_rand=0):
    from gymothelloenv_amd import VecOthelloEnv
    return VecOthelloEnv(E, board_size=n, sudden_death_on_invalid_move=sd, num_disk_as_reward=dr,
                         auto_reset=auto, seed=seed, env_id_base=id_base, initial_rand_steps=init_rand,
                         device="cuda:0")


def get_state_np(env):
    b, m, lg = env.get_state()
    return np_u64(b), m.cpu().numpy().view(np.uint16), np_u64(lg)


def test_kat(torch_cuda, golden_dir):
    torch = torch_cuda
    kat = json.load(open(os.path.join(golden_dir, "kat.json")))
    for n in SIZES:
        k = kat[str(n)]
        env = make_env(torch, 3, n)
        b, m, lg = get_state_np(env)
        W = oracle.nwords(n)
        for e in range(3):
            assert list(b[e, :W]) == k["black"] and list(b[e, W:]) == k["white"]
            moves = [a for a in range(n * n) if (int(lg[e, a // 64]) >> (a % 64)) & 1]
            assert moves == k["black_moves"]
        env.step(torch.full((3,), k["black_moves"][0], dtype=torch.int32))
        _, _, lg = get_state_np(env)
        moves = [a for a in range(n * n) if (int(lg[0, a // 64]) >> (a % 64)) & 1]
        assert moves == k["white_moves_after_lowest"]


@pytest.mark.parametrize("n", SIZES)
def test_step_matches_reference_golden(torch_cuda, golden_dir, n):
    """Every ply the reference recorded, stepped on the GPU from its pre-state."""
    torch = torch_cuda
    t = dict(np.load(os.path.join(golden_dir, "traj_N%d.npz" % n)))
    for ci, (sd, dr) in enumerate(t["combos"]):
        sel = t["combo"] == ci
        E = int(sel.sum())
        env = make_env(torch, E, n, sd=bool(sd), dr=bool(dr))
        env.set_state(t64(torch, np.concatenate([t["prev_black"][sel], t["prev_white"][sel]], axis=1)),
                      torch.from_numpy(oracle.meta_from(t["prev_turn"][sel]).view(np.int16)).cuda(),
                      t64(torch, t["prev_legal"][sel]))
        _, rew, dones, _ = env.step(torch.from_numpy(t["action"][sel]).cuda())
        b, m, lg = get_state_np(env)
        np.testing.assert_array_equal(b, np.concatenate([t["black"][sel], t["white"][sel]], axis=1))
        np.testing.assert_array_equal(lg, t["legal"][sel])
        np.testing.assert_array_equal(rew.cpu().numpy(), t["reward"][sel])
        np.testing.assert_array_equal(dones.cpu().numpy(), t["done"][sel])
        np.testing.assert_array_equal(np.where(m & 1, 1, -1), t["turn"][sel])
        wc = (m >> 2) & 3
        np.testing.assert_array_equal(np.where(wc == 1, 1, np.where(wc == 2, -1, 0)), t["winner"][sel])
        env.close()


@pytest.mark.parametrize("n", [4, 5, 8, 10, 16])
def test_games_in_lockstep(torch_cuda, golden_dir, n):
    """All recorded games of a combo advance together from reset, one GPU step
    per ply; finished games are masked with an (ignored) action."""
    torch = torch_cuda
    t = dict(np.load(os.path.join(golden_dir, "traj_N%d.npz" % n)))
    for ci, (sd, dr) in enumerate(t["combos"]):
        games = np.unique(t["game"][t["combo"] == ci])
        env = make_env(torch, len(games), n, sd=bool(sd), dr=bool(dr))
        idx = [np.flatnonzero((t["combo"] == ci) & (t["game"] == g)) for g in games]
        for p in range(max(len(i) for i in idx)):
            acts = np.array([t["action"][i[p]] if p < len(i) else 0 for i in idx], dtype=np.int32)
            _, rew, dn, _ = env.step(torch.from_numpy(acts).cuda())
            b, _, lg = get_state_np(env)
            rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
            for gi, i in enumerate(idx):
                if p < len(i):
                    k = i[p]
                    assert rew[gi] == t["reward"][k] and dn[gi] == t["done"][k]
                    assert list(b[gi]) == list(t["black"][k]) + list(t["white"][k])
                    assert list(lg[gi]) == list(t["legal"][k])
                else:  # past the end: stepping a terminated game is a no-op reporting done
                    assert dn[gi] == 1 and rew[gi] == 0


@pytest.mark.parametrize("n,E,plies", [(8, 65536, 130), (6, 16384, 80), (10, 8192, 200), (16, 1024, 260),
                                        (8, 1, 150), (8, 777, 100), (12, 333, 180)])
def test_random_rollout_replays_on_oracle(torch_cuda, n, E, plies):
    """Config 2 / 5: on-device random play with auto-reset; every action, reward,
    done, the final state and the W/D/L tally equal the oracle's replay."""
    torch = torch_cuda
    env = make_env(torch, E, n, auto=True, seed=7)
    acts, rews, dones = env.step_policy("random", n_plies=plies)
    b, m, lg = get_state_np(env)
    wdl = env.counts().cpu().numpy()
    s = oracle.reset(n, E)
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, False, True), 0, plies, seed=7)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(wdl, owdl)
    assert owdl.sum() >= E  # at least one finished game per board (ragged E: blocks past E store nothing)


@pytest.mark.parametrize("n,policy,sd,dr,auto,init_rand",
                         [(4, "random", True, True, True, 0), (5, "random", False, True, True, 4),
                          (7, "random", True, False, False, 0), (8, "random", False, False, True, 6),
                          (4, "greedy", True, True, True, 2), (7, "greedy", False, False, True, 6),
                          (5, "greedy", True, False, False, 4),
                          # multi-word boards: the FillsW engine (BB<W> ray tables + fills)
                          (9, "random", False, True, True, 4), (10, "greedy", True, False, True, 6),
                          (11, "random", True, True, False, 0), (12, "greedy", False, False, True, 4),
                          (14, "random", True, False, True, 2), (16, "random", False, True, True, 0),
                          (16, "greedy", True, False, True, 4)])
def test_fills_engine_flag_combinations(torch_cuda, n, policy, sd, dr, auto, init_rand):
    """The fills engine (flips from the legal scan carried across plies) under
    every flag combination, with and without auto-reset and random openings:
    identical to the oracle's replay ply by ply."""
    torch = torch_cuda
    # the oracle's greedy simulates every candidate move: fewer boards for the big boards' greedy cases
    E, plies = (1024 if policy == "greedy" and n >= 12 else 4096), 90
    env = make_env(torch, E, n, sd=sd, dr=dr, auto=auto, seed=5, init_rand=init_rand)
    env.reset()
    acts, rews, dones = env.step_policy(policy, n_plies=plies)
    b, m, lg = get_state_np(env)
    s = oracle.reset_openings(n, E, 5, 0, 0, init_rand) if init_rand else oracle.reset(n, E)
    pid = 0 if policy == "random" else 1
    oa, orw, od, owdl = oracle.rollout(s, flags_of(sd, dr, auto), pid, plies, seed=5, initial_rand_steps=init_rand)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)


@pytest.mark.parametrize("n", [6, 8, 10, 13])
def test_random_rollout_with_boards_loaded_terminated(torch_cuda, n):
    """k_play_rand's (and k_play_rand_w's) fallback: waves holding a board that was loaded
    terminated (set_state) run the generic ply loop; that board reports
    action -1 / done 1 every ply and is never reset (oth_step_policy's
    semantics), every other board of the wave plays on.  Equal to the oracle."""
    torch = torch_cuda
    E, plies = 4096, 70
    env = make_env(torch, E, n, auto=True, seed=13)
    env.step_policy("random", n_plies=9)
    b, m, lg = get_state_np(env)
    m = m.copy()
    m[::300] |= 2  # terminated (winner bits 0: a draw) in a few waves
    env.set_state(t64(torch, b), torch.from_numpy(m.view(np.int16)).cuda(), t64(torch, lg))
    env.counts(reset=True)
    acts, rews, dones = env.step_policy("random", n_plies=plies)
    s = oracle.State(n, E)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, False, True), 0, plies, seed=13, ply0=9)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    b2, m2, lg2 = get_state_np(env)
    np.testing.assert_array_equal(b2, s.boards)
    np.testing.assert_array_equal(m2, s.meta)
    np.testing.assert_array_equal(lg2, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)
    assert (oa[:, ::300] == -1).all()


def test_rollout_split_over_launches_is_identical(torch_cuda):
    """K plies in one launch == K single-ply launches (state round-trips HBM)."""
    torch = torch_cuda
    a = make_env(torch, 4096, 8, auto=True, seed=3)
    b = make_env(torch, 4096, 8, auto=True, seed=3)
    acts_a, _, _ = a.step_policy("random", n_plies=90)
    acts_b = torch.cat([b.step_policy("random", n_plies=1)[0] for _ in range(90)])
    assert torch.equal(acts_a, acts_b)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("n,init_rand", [(8, 10), (6, 4), (10, 6)])
def test_greedy_rollout_replays_on_oracle(torch_cuda, n, init_rand):
    """Config 3: greedy vs greedy after Philox random openings (0..init_rand plies)."""
    torch = torch_cuda
    E, plies = 2048, 140
    env = make_env(torch, E, n, auto=True, seed=11, init_rand=init_rand)
    env.reset()
    acts, rews, dones = env.step_policy("greedy", n_plies=plies)
    b, m, lg = get_state_np(env)
    s = oracle.reset_openings(n, E, 11, 0, 0, init_rand)
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, False, True), 1, plies, seed=11,
                                       initial_rand_steps=init_rand)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)


@pytest.mark.parametrize("n,policy,init_rand,plies", [(8, "greedy", 10, 140), (6, "random", 0, 80),
                                                      (10, "random", 0, 200)])
def test_configs_at_stated_size_replay_on_oracle(torch_cuda, n, policy, init_rand, plies):
    """Configs 3 and 5 at their stated 65,536 boards (BASELINE.json configs[2],
    configs[4]): greedy vs greedy after 0..10-ply random openings at 8x8, random
    play at 6x6 and 10x10; every action, reward, done, the final state and the
    W/D/L tally equal the oracle's replay (run on host threads)."""
    torch = torch_cuda
    E = 65536
    env = make_env(torch, E, n, auto=True, seed=21, init_rand=init_rand)
    env.reset()
    acts, rews, dones = env.step_policy(policy, n_plies=plies)
    b, m, lg = get_state_np(env)
    wdl = env.counts().cpu().numpy()
    s = oracle.reset_openings(n, E, 21, 0, 0, init_rand) if init_rand else oracle.reset(n, E)
    pid = 0 if policy == "random" else 1
    oa, orw, od, owdl = oracle.rollout_parallel(s, flags_of(True, False, True), pid, plies, seed=21,
                                                initial_rand_steps=init_rand)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(wdl, owdl)
    assert owdl.sum() >= E


@pytest.mark.parametrize("n", SIZES)
def test_greedy_actions_match_reference(torch_cuda, golden_dir, n):
    torch = torch_cuda
    g = np.load(os.path.join(golden_dir, "greedy.npz"))
    b, w, t, a = g["N%d_black" % n], g["N%d_white" % n], g["N%d_turn" % n], g["N%d_action" % n]
    env = make_env(torch, len(a), n)
    env.set_state(t64(torch, np.concatenate([b, w], axis=1)),
                  torch.from_numpy(oracle.meta_from(t).view(np.int16)).cuda())
    env.set_player_turn(1, mask=torch.from_numpy((t == 1).astype(np.uint8)).cuda())
    env.set_player_turn(-1, mask=torch.from_numpy((t == -1).astype(np.uint8)).cuda())
    np.testing.assert_array_equal(env.greedy_actions().cpu().numpy(), a)


def legal_bool(legal, n):
    a = np.arange(n * n)
    return ((legal[:, a // 64] >> (a % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)


@pytest.mark.parametrize("n", SIZES)
def test_external_steps_with_invalid_actions(torch_cuda, n):
    """Random external actions (legal, illegal, out of range) in all flag combos,
    with auto-reset, against the oracle for 2*N*N plies (N*N + 20 above 10x10: past every first game)."""
    torch = torch_cuda
    E = 1024
    rng = np.random.RandomState(n)
    plies = 2 * n * n if n <= 10 else n * n + 20  # past the first games' ends and auto-resets
    for sd in (True, False):
        for dr in (False, True):
            env = make_env(torch, E, n, sd=sd, dr=dr, auto=True, seed=5)
            s = oracle.reset(n, E)
            wdl = np.zeros(3, dtype=np.int64)
            for p in range(plies):
                lb = legal_bool(s.legal, n)
                pick = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
                wild = (rng.rand(E) < 0.05) | ~lb.any(axis=1)
                acts = np.where(wild, rng.randint(-2, n * n + 2, size=E), pick).astype(np.int32)
                orw, od, _ = oracle.step(s, flags_of(sd, dr, True), acts, seed=5, ply=p, wdl=wdl)
                _, rew, dn, _ = env.step(torch.from_numpy(acts).cuda(), observe=False)
                np.testing.assert_array_equal(rew.cpu().numpy(), orw)
                np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
            b, m, lg = get_state_np(env)
            np.testing.assert_array_equal(b, s.boards)
            np.testing.assert_array_equal(m, s.meta)
            np.testing.assert_array_equal(lg, s.legal)
            np.testing.assert_array_equal(env.counts().cpu().numpy(), wdl)


@pytest.mark.parametrize("n", [6, 8])
def test_observations_match_reference(torch_cuda, golden_dir, n):
    torch = torch_cuda
    o = np.load(os.path.join(golden_dir, "obs.npz"))
    E = len(o["N%d_turn" % n])
    env = make_env(torch, E, n)
    env.set_state(t64(torch, np.concatenate([o["N%d_black" % n], o["N%d_white" % n]], axis=1)),
                  torch.from_numpy(oracle.meta_from(o["N%d_turn" % n]).view(np.int16)).cuda(),
                  t64(torch, o["N%d_legal" % n]))
    for dt in (torch.int8, torch.int32, torch.int64, torch.float32, torch.float64):
        np.testing.assert_array_equal(env.observe("board", dt).cpu().numpy(), o["N%d_obs" % n])
        np.testing.assert_array_equal(env.observe("board_legal", dt).cpu().numpy(), o["N%d_obs2" % n])
        np.testing.assert_array_equal(env.observe("make_state", dt).cpu().numpy(), o["N%d_make_state" % n])
    ab = env.observe("absolute", torch.int64).cpu().numpy()
    W = oracle.nwords(n)
    bl = o["N%d_black" % n]
    for e in range(0, E, 97):
        for a in range(n * n):
            isb = (int(bl[e, a // 64]) >> (a % 64)) & 1
            assert ab[e].ravel()[a] == (-1 if isb else (1 if (int(o["N%d_white" % n][e, a // 64]) >> (a % 64)) & 1
                                                         else 0))
    assert W >= 1


@pytest.mark.parametrize("n", SIZES)
def test_stateless_legal_moves(torch_cuda, n):
    torch = torch_cuda
    from gymothelloenv_amd import legal_moves
    rng = np.random.RandomState(100 + n)
    E, W = 4096, oracle.nwords(n)
    cells = rng.randint(0, 3, size=(E, n * n))
    mover = np.zeros((E, W), dtype=np.uint64)
    opp = np.zeros((E, W), dtype=np.uint64)
    for a in range(n * n):
        mover[:, a // 64] |= (cells[:, a] == 1).astype(np.uint64) << np.uint64(a % 64)
        opp[:, a // 64] |= (cells[:, a] == 2).astype(np.uint64) << np.uint64(a % 64)
    out = legal_moves(n, t64(torch, mover), t64(torch, opp))
    np.testing.assert_array_equal(np_u64(out), oracle.legal(n, mover, opp))


def test_sharding_is_invisible(torch_cuda):
    """Two shards (env_id_base 0 and E/2) reproduce one unsharded handle."""
    torch = torch_cuda
    E = 8192
    whole = make_env(torch, E, 8, auto=True, seed=21)
    lo = make_env(torch, E // 2, 8, auto=True, seed=21, id_base=0)
    hi = make_env(torch, E // 2, 8, auto=True, seed=21, id_base=E // 2)
    aw, _, _ = whole.step_policy("random", n_plies=150)
    al, _, _ = lo.step_policy("random", n_plies=150)
    ah, _, _ = hi.step_policy("random", n_plies=150)
    assert torch.equal(aw, torch.cat([al, ah], dim=1))
    assert torch.equal(whole.counts(), lo.counts() + hi.counts())


def test_full_size_invariants(torch_cuda):
    """1,048,576 boards (config 4's global size on one GPU), 400 plies: structural
    invariants that need no oracle -- colours disjoint, legal squares empty,
    finished games == tally, every board finished >= 5 games."""
    torch = torch_cuda
    E = 1 << 20
    env = make_env(torch, E, 8, auto=True, seed=99)
    _, _, dones = env.step_policy("random", n_plies=400, record=True)
    b, m, lg = env.get_state()
    assert int((b[:, 0] & b[:, 1]).count_nonzero()) == 0
    assert int((lg[:, 0] & (b[:, 0] | b[:, 1])).count_nonzero()) == 0
    wdl = env.counts()
    assert int(wdl.sum()) == int(dones.sum())
    assert int(dones.sum(0).min()) >= 5
    frac = (wdl.double() / wdl.sum()).cpu().numpy()
    assert 0.43 < frac[0] < 0.49 and 0.03 < frac[1] < 0.06 and 0.47 < frac[2] < 0.53


def test_config4_shard_replays_on_oracle(torch_cuda):
    """Config 4's per-rank workload at its real global ids: rank 7 of 8 over
    1,048,576 boards (131,072 boards, env_id_base 917,504; the bench's weak-scaling
    shard), 100 plies of random play with auto-reset (k_play_rand<8> at two waves
    per SIMD), replayed by the oracle keyed by the same global ids (the
    harnesses' W/D/L, ppo_run_self_play.py:432-441): actions, rewards, dones,
    final state and W/D/L equal."""
    torch = torch_cuda
    from gymothelloenv_amd.distributed import ShardedVecOthelloEnv
    env = ShardedVecOthelloEnv(1 << 20, rank=7, world=8, board_size=8, auto_reset=True, seed=0, device="cuda:0")
    assert env.num_envs == 131072 and env.env_id_base == 917504
    env.reset()
    acts, rews, dones = env.step_policy("random", n_plies=100)
    s = oracle.reset(8, 131072)
    oa, orw, od, owdl = oracle.rollout_parallel(s, flags_of(True, False, True), 0, 100, seed=0, id_base=917504)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    b, m, lg = get_state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)
    assert owdl.sum() > 131072  # every board finished at least one game


@pytest.mark.parametrize("n", [6, 8, 10, 16])
def test_count_disks_batched_matches_oracle(torch_cuda, n):
    """count_disks (othello.py:468-471) of every board (k_count) on mid-game and
    finished positions equals the oracle's, whose count is pinned to the
    reference's disk-count rewards (test_oracle_golden)."""
    torch = torch_cuda
    E = 20011
    env = make_env(torch, E, n, auto=False, seed=21)
    for plies in (n * n // 3, n * n):  # mid-game, then most games over (boards kept terminated)
        env.step_policy("random", n_plies=plies, record=False)
        b, m, lg = get_state_np(env)
        s = oracle.State(n, E)
        s.boards[:], s.meta[:], s.legal[:] = b, m, lg
        np.testing.assert_array_equal(env.count_disks().cpu().numpy(), oracle.count_disks(s))


def test_state_dict_roundtrip(torch_cuda):
    torch = torch_cuda
    a = make_env(torch, 1000, 8, auto=True, seed=4)
    a.step_policy("random", n_plies=33)
    sd = a.state_dict()
    b = make_env(torch, 1000, 8, auto=True, seed=4)
    b.load_state_dict(sd)
    x, _, _ = a.step_policy("random", n_plies=50)
    y, _, _ = b.step_policy("random", n_plies=50)
    assert torch.equal(x, y)


@pytest.mark.parametrize("n", [6, 8])
def test_vs_greedy_matches_reference(torch_cuda, golden_dir, n):
    """Device OthelloEnv (oth_reset_vs / oth_step_vs, greedy opponent) replays the
    reference's OthelloEnv games in lockstep (finished games are no-ops)."""
    torch = torch_cuda
    v = np.load(os.path.join(golden_dir, "vs_greedy.npz"))
    W = oracle.nwords(n)
    for ci, (prot, sd, dr) in enumerate(v["N%d_combos" % n]):
        sel = v["N%d_combo" % n] == ci
        games = np.unique(v["N%d_game" % n][sel])
        idx = [np.flatnonzero(sel & (v["N%d_game" % n] == g)) for g in games]
        env = make_env(torch, len(games), n, sd=bool(sd), dr=bool(dr))
        env.reset_vs("greedy", protagonist=int(prot))
        b, _, _ = get_state_np(env)
        n_games = len(games)
        np.testing.assert_array_equal(b[:, :W], v["N%d_start_black" % n][ci * n_games:(ci + 1) * n_games])
        np.testing.assert_array_equal(b[:, W:], v["N%d_start_white" % n][ci * n_games:(ci + 1) * n_games])
        for p in range(max(len(i) for i in idx)):
            acts = np.array([v["N%d_action" % n][i[p]] if p < len(i) else 0 for i in idx], dtype=np.int32)
            _, rew, dn, plies = env.step_vs(torch.from_numpy(acts).cuda(), "greedy", observe=False)
            b, m, _ = get_state_np(env)
            rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
            for gi, i in enumerate(idx):
                if p < len(i):
                    k = i[p]
                    assert rew[gi] == v["N%d_reward" % n][k] and bool(dn[gi]) == bool(v["N%d_done" % n][k])
                    assert list(b[gi, :W]) == list(v["N%d_black" % n][k])
                    assert list(b[gi, W:]) == list(v["N%d_white" % n][k])
                    assert (1 if m[gi] & 1 else -1) == v["N%d_turn" % n][k]
                else:
                    assert dn[gi] and rew[gi] == 0


@pytest.mark.parametrize("n,opp,init_rand", [(8, "random", 0), (8, "random", 10), (8, "greedy", 6), (6, "greedy", 0),
                                              (10, "random", 4)])
def test_vs_rollout_replays_on_oracle(torch_cuda, n, opp, init_rand):
    """Mixed protagonist colours, random openings and auto-reset: every call's
    rewards / dones / plies, the final state and the W/D/L tally equal the oracle."""
    torch = torch_cuda
    E, calls = 4096, 80
    pol = 0 if opp == "random" else 1
    prot = np.where(np.arange(E) % 3 == 0, -1, 1).astype(np.int8)
    env = make_env(torch, E, n, auto=True, seed=13, init_rand=init_rand)
    env.reset_vs(opp, protagonist=torch.from_numpy(prot))
    flags = flags_of(True, False, True)
    s = oracle.reset_vs(n, E, flags, pol, 0, seed=13, initial_rand_steps=init_rand, prot=prot)
    b, m, lg = get_state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    rng = np.random.RandomState(n)
    wdl = np.zeros(3, dtype=np.int64)
    for c in range(1, calls + 1):
        lb = legal_bool(s.legal, n)
        pick = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
        acts = np.where((rng.rand(E) < 0.02) | ~lb.any(axis=1), rng.randint(-1, n * n, size=E), pick).astype(np.int32)
        orw, od, opl = oracle.step_vs(s, flags, pol, c, acts, seed=13, initial_rand_steps=init_rand, prot=prot, wdl=wdl)
        _, rew, dn, plies = env.step_vs(torch.from_numpy(acts).cuda(), opp, observe=False)
        np.testing.assert_array_equal(rew.cpu().numpy(), orw)
        np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
        np.testing.assert_array_equal(plies.cpu().numpy(), opl)
    b, m, lg = get_state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), wdl)


@pytest.mark.parametrize("n,opp,sd,dr,auto", [(8, "random", False, True, True), (8, "greedy", False, False, False),
                                              (8, "random", True, True, False), (6, "greedy", False, True, True),
                                              (10, "greedy", False, True, True)])
def test_vs_flag_combinations_on_oracle(torch_cuda, n, opp, sd, dr, auto):
    """OthelloEnv.step on the device (k_step_vs1 on one-word boards, k_step_vs on
    10x10) with the other env flags: invalid protagonist actions without sudden
    death (the turn passes, othello.py:417-427), disk-count rewards (:446-459)
    negated after opponent plies (:200), and boards left terminated without
    auto-reset (a step on them reports done); rewards / dones / plies / state /
    protagonist W/D/L equal the oracle's every call."""
    torch = torch_cuda
    E, calls = 2048, 60
    pol = 0 if opp == "random" else 1
    prot = np.where(np.arange(E) % 3 == 0, -1, 1).astype(np.int8)
    env = make_env(torch, E, n, sd=sd, dr=dr, auto=auto, seed=19, init_rand=4)
    env.reset_vs(opp, protagonist=torch.from_numpy(prot))
    flags = flags_of(sd, dr, auto)
    s = oracle.reset_vs(n, E, flags, pol, 0, seed=19, initial_rand_steps=4, prot=prot)
    rng = np.random.RandomState(100 + n)
    wdl = np.zeros(3, dtype=np.int64)
    for c in range(1, calls + 1):
        lb = legal_bool(s.legal, n)
        pick = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
        acts = np.where((rng.rand(E) < 0.05) | ~lb.any(axis=1), rng.randint(-1, n * n, size=E), pick).astype(np.int32)
        orw, od, opl = oracle.step_vs(s, flags, pol, c, acts, seed=19, initial_rand_steps=4, prot=prot, wdl=wdl)
        _, rew, dn, plies = env.step_vs(torch.from_numpy(acts).cuda(), opp, observe=False)
        np.testing.assert_array_equal(rew.cpu().numpy(), orw)
        np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
        np.testing.assert_array_equal(plies.cpu().numpy(), opl)
    b, m, lg = get_state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), wdl)
    if not auto:
        assert (m & 2).any(), "no board finished: the no-auto-reset path is untested"


@pytest.mark.parametrize("n,depth", [(6, 1), (6, 2), (6, 3), (8, 1), (8, 2), (8, 3), (6, 4), (6, 5), (8, 4),
                                     (4, 6), (4, 7), (4, 8), (4, 9), (4, 10), (5, 6), (5, 7), (6, 6), (8, 6)])
def test_maximin_actions_match_reference(torch_cuda, golden_dir, n, depth):
    """MaxiMinPolicy(depth).get_action (simple_policies.py:98-163) on device;
    depth >= 4 runs the explicit-stack search (maximin_search); depths 6..10
    on the late positions of maximin_deeper.npz."""
    torch = torch_cuda
    g = np.load(os.path.join(golden_dir, "maximin.npz" if depth <= 3 else
                             ("maximin_deep.npz" if depth <= 5 else "maximin_deeper.npz")))
    k = "N%d_d%d_" % (n, depth)
    b, w, t, a = g[k + "black"], g[k + "white"], g[k + "turn"], g[k + "action"]
    env = make_env(torch, len(a), n)
    env.set_state(t64(torch, np.concatenate([b, w], axis=1)),
                  torch.from_numpy(oracle.meta_from(t).view(np.int16)).cuda())
    env.set_player_turn(1, mask=torch.from_numpy((t == 1).astype(np.uint8)).cuda())
    env.set_player_turn(-1, mask=torch.from_numpy((t == -1).astype(np.uint8)).cuda())
    np.testing.assert_array_equal(env.policy_actions("maximin%d" % depth).cpu().numpy(), a)


@pytest.mark.parametrize("n,policy,pid", [(8, "maximin2", 3), (6, "maximin3", 4), (10, "maximin2", 3),
                                          (6, "maximin4", 5), (5, "maximin5", 6)])
def test_maximin_rollout_replays_on_oracle(torch_cuda, n, policy, pid):
    torch = torch_cuda
    E, plies = (256 if pid >= 5 else 512), 70  # the oracle's search at depth >= 4 is the slow side
    env = make_env(torch, E, n, auto=True, seed=23, init_rand=8)
    env.reset()
    acts, rews, dones = env.step_policy(policy, n_plies=plies)
    b, m, lg = get_state_np(env)
    s = oracle.reset_openings(n, E, 23, 0, 0, 8)
    oa, orw, od, owdl = oracle.rollout(s, flags_of(True, False, True), pid, plies, seed=23, initial_rand_steps=8)
    np.testing.assert_array_equal(acts.cpu().numpy(), oa)
    np.testing.assert_array_equal(rews.cpu().numpy(), orw)
    np.testing.assert_array_equal(dones.cpu().numpy(), od)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)


def test_vs_maximin_opponent_on_oracle(torch_cuda):
    torch = torch_cuda
    n, E, calls = 8, 1024, 40
    prot = np.where(np.arange(E) % 2 == 0, -1, 1).astype(np.int8)
    env = make_env(torch, E, n, auto=True, seed=29, init_rand=4)
    env.reset_vs("maximin2", protagonist=torch.from_numpy(prot))
    s = oracle.reset_vs(n, E, flags_of(True, False, True), 3, 0, seed=29, initial_rand_steps=4, prot=prot)
    rng = np.random.RandomState(1)
    for c in range(1, calls + 1):
        lb = legal_bool(s.legal, n)
        acts = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
        orw, od, opl = oracle.step_vs(s, flags_of(True, False, True), 3, c, acts, seed=29, initial_rand_steps=4,
                                      prot=prot)
        _, rew, dn, plies = env.step_vs(torch.from_numpy(acts).cuda(), "maximin2", observe=False)
        np.testing.assert_array_equal(rew.cpu().numpy(), orw)
        np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
        np.testing.assert_array_equal(plies.cpu().numpy(), opl)
    b, m, lg = get_state_np(env)
    np.testing.assert_array_equal(b, s.boards)


def _obs_np(n, boards, meta, legal, layout):
    """numpy restatement of get_observation / make_state / board_state for the
    observation kernels (othello.py:257,363-376; util.py:48-74)."""
    W = oracle.nwords(n)
    sq = np.arange(n * n)

    def bits(words):
        return ((words[:, sq // 64] >> (sq % 64).astype(np.uint64)) & np.uint64(1)).astype(np.int64)

    b, w, lg = bits(boards[:, :W]), bits(boards[:, W:]), bits(legal)
    tw = (meta.astype(np.int64) & 1).astype(bool)[:, None]
    E = len(meta)
    if layout == "absolute":
        return (w - b).reshape(E, n, n)
    if layout == "legal":
        return lg.reshape(E, n, n)
    mover = np.where(tw, w - b, b - w)
    if layout == "board":
        return mover.reshape(E, n, n)
    if layout == "board_legal":
        return np.stack([mover, lg], 1).reshape(E, 2, n, n)
    ms_legal = np.where(lg.sum(1, keepdims=True) > 1, lg, 0)
    return np.stack([b, w, np.broadcast_to(tw.astype(np.int64), b.shape), ms_legal], 1).reshape(E, 4, n, n)


def _host(o):
    """An observation as numpy; bfloat16 (absent from numpy) as float32 after
    checking its bit patterns are exactly bfloat16's -1 / 0 / +1."""
    import torch
    if o.dtype == torch.bfloat16:
        bits = o.view(torch.int16).cpu().numpy()
        assert np.isin(bits, [0, 0x3F80, 0xBF80 - 0x10000]).all()
        return o.float().cpu().numpy()
    return o.cpu().numpy()


@pytest.mark.parametrize("n", [4, 5, 7, 8, 10, 16])
def test_observation_kernels_every_layout_and_alignment(torch_cuda, n):
    """Vector-store quad kernel (N*N % 4 == 0, aligned out) and the scalar kernel
    (odd N, or an out pointer off the 4-element alignment) write the same values
    as a numpy restatement, for every layout and dtype, on mid-game boards."""
    torch = torch_cuda
    E = 1000
    env = make_env(torch, E, n, auto=True, seed=5)
    env.step_policy("random", n_plies=n * n // 2 + 3, record=False)
    b, m, lg = get_state_np(env)
    for layout in ("board", "board_legal", "make_state", "absolute", "legal"):
        want = _obs_np(n, b, m, lg, layout)
        for dt in (torch.int8, torch.int32, torch.int64, torch.float32, torch.float64, torch.bfloat16):
            got = env.observe(layout, dt)
            np.testing.assert_array_equal(_host(got), want, err_msg="%s %s" % (layout, dt))
            buf = torch.empty(want.size + 1, dtype=dt, device=got.device)
            off = buf[1:].view(want.shape)  # base one element past the vector alignment
            env.observe(layout, dt, out=off)
            np.testing.assert_array_equal(_host(off), want, err_msg="unaligned %s %s" % (layout, dt))
    np.testing.assert_array_equal(env.legal_actions().cpu().numpy(),
                                  _obs_np(n, b, m, lg, "legal").reshape(E, n * n).astype(bool))


@pytest.mark.parametrize("n,E", [(8, 65536), (8, 262144), (6, 100003), (10, 70000)])
def test_observation_kernels_at_size(torch_cuda, n, E):
    """k_observe_w's wave shapes (16 boards per wave below 262,144 boards, 64
    from there up to 384 MiB of output) at the configs' sizes and ragged E:
    int64 BOARD and f32 MAKE_STATE equal the numpy restatement."""
    torch = torch_cuda
    env = make_env(torch, E, n, auto=True, seed=8)
    env.step_policy("random", n_plies=n * n // 2 + 1, record=False)
    b, m, lg = get_state_np(env)
    for layout, dt in (("board", torch.int64), ("make_state", torch.float32), ("legal", torch.int8),
                       ("make_state", torch.int8), ("make_state", torch.bfloat16)):
        np.testing.assert_array_equal(_host(env.observe(layout, dt)), _obs_np(n, b, m, lg, layout),
                                      err_msg="%s %s" % (layout, dt))


@pytest.mark.parametrize("n,E", [(8, 262147), (6, 300001)])
def test_observation_large_launches_every_layout_and_dtype(torch_cuda, n, E):
    """From 262,144 boards k_observe_w takes 64 boards a wave (and 4-KiB output
    regions past 384 MiB of output: the next test): every layout and dtype at
    ragged E equal the numpy restatement."""
    torch = torch_cuda
    env = make_env(torch, E, n, auto=True, seed=12)
    env.step_policy("random", n_plies=n * n // 2 + 3, record=False)
    b, m, lg = get_state_np(env)
    for layout in ("board", "board_legal", "make_state", "absolute", "legal"):
        want = _obs_np(n, b, m, lg, layout)
        for dt in (torch.int8, torch.int32, torch.int64, torch.float32, torch.float64, torch.bfloat16):
            got = _host(env.observe(layout, dt))
            np.testing.assert_array_equal(got, want.astype(got.dtype), err_msg="%s %s" % (layout, dt))


def test_observation_beyond_384_mib_equals_small_launches(torch_cuda):
    """Past 384 MiB of output k_observe_w takes as many boards per wave as fill
    about 4 KiB (make_state f32 and board_legal f64: 4, the int64 board: 8);
    1,048,579 8x8 boards: slices of each big observation equal the observation
    of the same boards from a 70,001-board handle (16 boards a wave, itself
    checked against numpy above)."""
    torch = torch_cuda
    E, n = 1048579, 8
    env = make_env(torch, E, n, auto=True, seed=21)
    env.step_policy("random", n_plies=37, record=False)
    b, m, lg = env.get_state()
    small = make_env(torch, 70001, n, auto=True, seed=21)
    for lay, dt in (("make_state", torch.float32), ("board", torch.int64), ("board_legal", torch.float64),
                    ("legal", torch.int8)):
        big = env.observe(lay, dt)
        for lo in (0, 500000, E - 70001):
            small.set_state(b[lo:lo + 70001], m[lo:lo + 70001], lg[lo:lo + 70001])
            assert torch.equal(big[lo:lo + 70001], small.observe(lay, dt)), "%s %s at %d" % (lay, dt, lo)
        del big
    small.close()
    env.close()


@pytest.mark.parametrize("n,opp", [(8, "random"), (6, "greedy")])
def test_protagonist_tally_matches_oracle_rewards(torch_cuda, n, opp):
    """counts_vs: {protagonist wins, draws, losses} of games step_vs finished,
    with mixed protagonist colours, equals run.py:100-130's count from the
    protagonist's final rewards (sign) replayed by the oracle."""
    torch = torch_cuda
    E, calls = 2048, 40
    env = make_env(torch, E, n, auto=True, seed=17, init_rand=2)
    prot = np.where(np.arange(E) % 3 == 0, 1, -1).astype(np.int8)
    pid = 0 if opp == "random" else 1
    env.reset_vs(opp, protagonist=torch.from_numpy(prot).cuda())
    s = oracle.reset_vs(n, E, flags_of(True, False, True), pid, 0, seed=17, initial_rand_steps=2, prot=prot)
    rng = np.random.RandomState(1)
    tally = np.zeros(3, dtype=np.int64)
    env.counts_vs(reset=True)
    for c in range(1, calls + 1):
        legal = s.legal[:, 0]
        acts = np.array([np.flatnonzero([(int(x) >> b) & 1 for b in range(n * n)])[0] if x else 0
                         for x in legal], dtype=np.int32)
        acts[rng.rand(E) < 0.05] = rng.randint(0, n * n)  # a few invalid moves: sudden-death losses
        _, r, d, _ = env.step_vs(torch.from_numpy(acts).cuda(), opponent=opp, observe=False)
        orw, od, _ = oracle.step_vs(s, flags_of(True, False, True), pid, c, acts, seed=17, initial_rand_steps=2,
                                    prot=prot)
        np.testing.assert_array_equal(r.cpu().numpy(), orw)
        np.testing.assert_array_equal(d.cpu().numpy(), od)
        fin = od.astype(bool)
        tally += [(orw[fin] > 0).sum(), (orw[fin] == 0).sum(), (orw[fin] < 0).sum()]
    np.testing.assert_array_equal(env.counts_vs().cpu().numpy(), tally)
    assert tally.sum() > 0 and tally[0] > 0 and tally[2] > 0


def test_greedy_vs_random_split_near_readme(torch_cuda):
    """Statistical sanity only (not a pin): greedy protagonist (black) against
    the random opponent over 65,536 device games lands near the README's
    61 / 5 / 34 row (README.md:46, 100 games there, so +-12 points)."""
    torch = torch_cuda
    E = 65536
    env = make_env(torch, E, 8, auto=True, seed=23)
    env.reset_vs("random", protagonist=-1)
    env.counts_vs(reset=True)
    for _ in range(200):
        acts = env.greedy_actions()
        env.step_vs(acts, opponent="random", observe=False)
    w, d, l = env.counts_vs().cpu().numpy().astype(float)
    tot = w + d + l
    assert tot > E
    assert abs(100 * w / tot - 61) < 12 and abs(100 * d / tot - 5) < 5 and abs(100 * l / tot - 34) < 12, (w, d, l)


@pytest.mark.parametrize("n,E", [(8, 70001), (6, 70001), (5, 1000), (8, 65536)])
def test_single_ply_kernels_both_ray_sources(torch_cuda, n, E):
    """The single-ply kernels (ply.hpp) compute their rays up to 65,536 boards
    and read the handle's LDS-staged table beyond: both equal the oracle for
    external actions (legal, illegal, out of range; both sudden-death modes)
    and for one-ply random play, ragged E included; a dones view at every byte
    offset, guarded on both sides against writes outside the view."""
    torch = torch_cuda
    rng = np.random.RandomState(E + n)
    for sd in (True, False):
        env = make_env(torch, E, n, sd=sd, auto=True, seed=9)
        s = oracle.reset(n, E)
        for p in range(6):
            lb = legal_bool(s.legal, n)
            pick = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
            wild = (rng.rand(E) < 0.1) | ~lb.any(axis=1)
            acts = np.where(wild, rng.randint(-2, n * n + 2, size=E), pick).astype(np.int32)
            orw, od, _ = oracle.step(s, flags_of(sd, False, True), acts, seed=9, ply=p)
            off = p % 4  # a dones view at every byte offset
            dbuf = torch.full((E + 4,), 7, dtype=torch.uint8, device="cuda")
            _, rew, dn, _ = env.step(torch.from_numpy(acts).cuda(), dones=dbuf[off:off + E], observe=False)
            np.testing.assert_array_equal(rew.cpu().numpy(), orw)
            np.testing.assert_array_equal(dn.view(torch.uint8).cpu().numpy(), od.astype(np.uint8))
            guard = dbuf.cpu().numpy()
            assert (guard[:off] == 7).all() and (guard[off + E:] == 7).all(), "dones written outside its view"
        b, m, lg = get_state_np(env)
        np.testing.assert_array_equal(b, s.boards)
        np.testing.assert_array_equal(m, s.meta)
        np.testing.assert_array_equal(lg, s.legal)
        # one-ply random launches from this state (ply counter 6)
        wdl0 = env.counts().cpu().numpy()
        acts = [env.step_policy("random", n_plies=1) for _ in range(3)]
        oa, orw, od, owdl = oracle.rollout(s, flags_of(sd, False, True), 0, 3, seed=9, ply0=6)
        np.testing.assert_array_equal(torch.cat([a[0] for a in acts]).cpu().numpy(), oa)
        np.testing.assert_array_equal(torch.cat([a[1] for a in acts]).cpu().numpy(), orw)
        np.testing.assert_array_equal(torch.cat([a[2] for a in acts]).cpu().numpy(), od)
        b, m, lg = get_state_np(env)
        np.testing.assert_array_equal(b, s.boards)
        np.testing.assert_array_equal(m, s.meta)
        np.testing.assert_array_equal(lg, s.legal)
        np.testing.assert_array_equal(env.counts().cpu().numpy() - wdl0, owdl)


@pytest.mark.parametrize("n,E,depth", [(8, 256, 3), (8, 128, 4), (6, 256, 5), (4, 1024, 8), (10, 48, 4),
                                       (8, 40, 5), (5, 300, 6), (8, 2049, 4), (6, 4096, 5),
                                       # above OTH_MM_NESTED_MAX_E (8,192): the explicit-stack subtrees
                                       (8, 8195, 4), (6, 8200, 4), (4, 9000, 7)])
def test_maximin_wave_matches_oracle(torch_cuda, n, E, depth):
    """MaxiMin of depth >= 3 on a wave per board (k_maximin_wave: the root's moves
    and replies over the lanes, maximin_node or maximin_value below) equals the oracle's search
    (simple_policies.py:98-163 restated) on mid-game and late positions, ragged
    E included; MaxiMin-2 (one lane per board) is unchanged.  The boards are
    independent, so large launches check their first and last 400 boards (the
    oracle's 8x8 depth-4 search takes ~15 ms a board)."""
    torch = torch_cuda
    env = make_env(torch, E, n, auto=True, seed=depth + n)
    idx = np.r_[0:400, E - 400:E] if E > 1600 else np.arange(E)
    for plies in (n * n // 3, n * n // 3):
        env.step_policy("random", n_plies=plies, record=False)
        b, m, lg = get_state_np(env)
        s = oracle.State(n, len(idx))
        s.boards[:], s.meta[:], s.legal[:] = b[idx], m[idx], lg[idx]
        got = env.policy_actions("maximin%d" % depth).cpu().numpy()
        np.testing.assert_array_equal(got[idx], oracle.maximin(s, depth))
        assert (got >= 0).any()


@pytest.mark.parametrize("n,E,plies,depth", [(6, 300, 24, 20), (4, 500, 5, 12), (8, 64, 52, 60)])
def test_maximin_any_depth_by_empty_squares(torch_cuda, n, E, plies, depth):
    """MaxiMin deeper than OTH_MAXIMIN_MAX_DEPTH, as the reference allows
    (simple_policies.py:101-103): on boards with at most 10 empty squares the
    search runs at the batch's largest empty-square count, which every deeper
    search equals (each level places a disc); equal to the oracle's search at
    the full depth.  Earlier in the game the call raises."""
    torch = torch_cuda
    env = make_env(torch, E, n, auto=False, seed=depth + n)
    with pytest.raises(ValueError, match="empty squares"):
        env.policy_actions("maximin%d" % depth)  # the start position: n*n - 4 > 10 empty squares
    env.step_policy("random", n_plies=plies, record=False)
    b, m, lg = get_state_np(env)
    s = oracle.State(n, E)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    got = env.policy_actions("maximin%d" % depth).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.maximin(s, depth))
    assert (got >= 0).any()


def test_maximin_leaf_budget_refuses_before_launch(torch_cuda):
    """oth_policy_actions refuses a MaxiMin call whose search is estimated above
    OTH_MAXIMIN_LEAF_BUDGET leaves (E x b^d) with a message naming the split,
    before anything is launched; a smaller batch of the same depth runs."""
    torch = torch_cuda
    from gymothelloenv_amd._lib import OthelloLibError
    env = make_env(torch, 65536, 8, auto=True, seed=1)
    with pytest.raises(OthelloLibError, match="split the boards"):
        env.policy_actions("maximin7")
    with pytest.raises(OthelloLibError, match="split the boards"):  # 100 searches per board
        env.step_policy("maximin5", n_plies=100, record=False)
    with pytest.raises(OthelloLibError, match="split the boards"):
        env.reset_vs("maximin7")
    small = make_env(torch, 2, 8, auto=True, seed=1)
    small.step_policy("random", n_plies=40, record=False)
    assert small.policy_actions("maximin5").shape == (2,)
