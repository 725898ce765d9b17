"""Pin the CPU oracle (oracle/othello_oracle.c) to the reference's own outputs.

The fixtures in tests/golden/ were produced by tests/golden/gen_golden.py, which
imports the reference othello.py / simple_policies.py / util.py.  Every
GPU parity test later compares the HIP path against this oracle, so this file
is what makes those comparisons mean "identical to the reference".
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle

SIZES = list(range(4, 17))


def load_traj(golden_dir, n):
    return dict(np.load(os.path.join(golden_dir, "traj_N%d.npz" % n)))


def decode_meta(meta):
    turn = np.where(meta & 1, 1, -1)
    term = (meta >> 1) & 1
    wc = (meta >> 2) & 3
    winner = np.where(wc == 1, 1, np.where(wc == 2, -1, 0))
    return turn, term, winner


def test_kat(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "kat.json")))
    for n in SIZES:
        k = kat[str(n)]
        s = oracle.reset(n, 1)
        W = oracle.nwords(n)
        assert list(s.boards[0, :W]) == k["black"]
        assert list(s.boards[0, W:]) == k["white"]
        moves = [a for a in range(n * n) if (int(s.legal[0, a // 64]) >> (a % 64)) & 1]
        assert moves == k["black_moves"]
        oracle.step(s, oracle.F_SUDDEN_DEATH, np.array([moves[0]]))
        moves2 = [a for a in range(n * n) if (int(s.legal[0, a // 64]) >> (a % 64)) & 1]
        assert moves2 == k["white_moves_after_lowest"]
        assert k["action_space_n"] == n * n


@pytest.mark.parametrize("n", SIZES)
def test_step_matches_reference_per_ply(golden_dir, n):
    """Each recorded ply, stepped from its recorded pre-state, reproduces the
    reference's post-state, possible_moves (incl. stale terminals), reward, done."""
    t = load_traj(golden_dir, n)
    combos = t["combos"]
    for ci, (sd, dr) in enumerate(combos):
        sel = t["combo"] == ci
        E = int(sel.sum())
        s = oracle.State(n, E)
        s.boards[:] = np.concatenate([t["prev_black"][sel], t["prev_white"][sel]], axis=1)
        s.meta[:] = oracle.meta_from(t["prev_turn"][sel])
        s.legal[:] = t["prev_legal"][sel]
        flags = (oracle.F_SUDDEN_DEATH if sd else 0) | (oracle.F_DISK_REWARD if dr else 0)
        rew, dones, errs = oracle.step(s, flags, t["action"][sel])
        assert errs == 0
        np.testing.assert_array_equal(s.boards, np.concatenate([t["black"][sel], t["white"][sel]], axis=1))
        np.testing.assert_array_equal(s.legal, t["legal"][sel])
        turn, term, winner = decode_meta(s.meta)
        np.testing.assert_array_equal(turn, t["turn"][sel])
        np.testing.assert_array_equal(term, t["done"][sel].astype(int))
        np.testing.assert_array_equal(winner, t["winner"][sel])
        np.testing.assert_array_equal(rew, t["reward"][sel])
        np.testing.assert_array_equal(dones, t["done"][sel])


@pytest.mark.parametrize("n", SIZES)
def test_count_disks_matches_reference_rewards(golden_dir, n):
    """oracle count_disks (othello.py:468-471) on every recorded post-ply board:
    the popcounts of the reference's own board, and -- on the terminal plies of
    the disk-reward runs that did not end by sudden death -- the reference's
    reward, which it computes from count_disks (:444-461: mover's minus the
    opponent's discs, N*N when the opponent has none)."""
    t = load_traj(golden_dir, n)
    E = len(t["action"])
    s = oracle.State(n, E)
    s.boards[:] = np.concatenate([t["black"], t["white"]], axis=1)
    s.meta[:] = oracle.meta_from(t["turn"])
    wb = oracle.count_disks(s)

    def pc(words):
        return np.array([sum(bin(int(x)).count("1") for x in row) for row in words])
    np.testing.assert_array_equal(wb[:, 0], pc(t["white"]))
    np.testing.assert_array_equal(wb[:, 1], pc(t["black"]))
    dr = t["combos"][t["combo"], 1].astype(bool)
    sudden = t["combos"][t["combo"], 0].astype(bool) & (t["reward"] == -n * n)
    sel = t["done"] & dr & ~sudden
    mover_white = t["prev_turn"][sel] == 1
    mine = np.where(mover_white, wb[sel, 0], wb[sel, 1])
    theirs = np.where(mover_white, wb[sel, 1], wb[sel, 0])
    want = np.where(theirs == 0, n * n, mine - theirs)
    assert sel.sum() > 0
    np.testing.assert_array_equal(t["reward"][sel], want)


@pytest.mark.parametrize("n", [4, 5, 8, 10, 16])
def test_whole_games_replay(golden_dir, n):
    """Replaying each game's action list from reset reproduces every ply."""
    t = load_traj(golden_dir, n)
    for ci, (sd, dr) in enumerate(t["combos"]):
        flags = (oracle.F_SUDDEN_DEATH if sd else 0) | (oracle.F_DISK_REWARD if dr else 0)
        games = np.unique(t["game"][t["combo"] == ci])
        for g in games:
            sel = np.flatnonzero((t["combo"] == ci) & (t["game"] == g))
            s = oracle.reset(n, 1)
            for i in sel:
                r, d, errs = oracle.step(s, flags, t["action"][i:i + 1])
                assert errs == 0
                assert r[0] == t["reward"][i] and d[0] == t["done"][i]
                assert list(s.boards[0]) == list(t["black"][i]) + list(t["white"][i])
                assert list(s.legal[0]) == list(t["legal"][i])
            # stepping again after the terminal ply is the reference's ValueError
            r, d, errs = oracle.step(s, flags, np.array([0]))
            assert errs == 1 and d[0] == 1 and r[0] == 0


def test_edge_cases_are_covered(golden_dir):
    """The fixtures exercise every terminal / pass path the reference has."""
    seen = {"double_pass": 0, "wipeout": 0, "sudden": 0, "invalid_pass": 0, "pass": 0}
    for n in SIZES:
        t = load_traj(golden_dir, n)
        nn = n * n
        for i in range(len(t["action"])):
            sd, dr = t["combos"][t["combo"][i]]
            a = int(t["action"][i])
            invalid = not ((int(t["prev_legal"][i][a // 64]) >> (a % 64)) & 1) if 0 <= a < nn else True
            if t["done"][i] and invalid and sd:
                seen["sudden"] += 1
            if invalid and not sd and not t["done"][i]:
                seen["invalid_pass"] += 1
            if not t["done"][i] and t["turn"][i] == t["prev_turn"][i]:
                seen["pass"] += 1
            full = sum(bin(int(x)).count("1") for x in (t["black"][i] | t["white"][i])) == nn
            if t["done"][i] and not invalid and not full:
                seen["double_pass"] += 1
            if t["done"][i] and dr and t["reward"][i] == nn:
                seen["wipeout"] += 1
    for k, v in seen.items():
        assert v > 0, k


@pytest.mark.parametrize("n", SIZES)
def test_greedy_matches_reference(golden_dir, n):
    g = np.load(os.path.join(golden_dir, "greedy.npz"))
    b, w, t, a = g["N%d_black" % n], g["N%d_white" % n], g["N%d_turn" % n], g["N%d_action" % n]
    s = oracle.State(n, len(a))
    s.boards[:] = np.concatenate([b, w], axis=1)
    s.meta[:] = oracle.meta_from(t)
    s.legal[:] = oracle.recompute_legal(s)
    np.testing.assert_array_equal(oracle.greedy(s), a)


@pytest.mark.parametrize("n", [6, 8])
def test_observations_match_reference(golden_dir, n):
    o = np.load(os.path.join(golden_dir, "obs.npz"))
    s = oracle.State(n, len(o["N%d_turn" % n]))
    s.boards[:] = np.concatenate([o["N%d_black" % n], o["N%d_white" % n]], axis=1)
    s.meta[:] = oracle.meta_from(o["N%d_turn" % n])
    s.legal[:] = o["N%d_legal" % n]
    obs, obs2, ms = oracle.observe(s)
    np.testing.assert_array_equal(obs, o["N%d_obs" % n])
    np.testing.assert_array_equal(obs2, o["N%d_obs2" % n])
    np.testing.assert_array_equal(ms, o["N%d_make_state" % n].astype(np.float32))
    assert (o["N%d_nlegal" % n] == 1).any()  # the single-legal-move quirk is exercised


def test_random_policy_distribution():
    """Philox random play: outcome split near the reference's (46/4/49 %)."""
    s = oracle.reset(8, 2000)
    _, _, dones, wdl = oracle.rollout(s, oracle.F_SUDDEN_DEATH, 0, 64, seed=0)
    assert wdl.sum() == 2000  # every 8x8 random game ends within 60 + passes <= 64 plies
    frac = wdl / wdl.sum()
    assert 0.40 < frac[0] < 0.52 and 0.02 < frac[1] < 0.08 and 0.43 < frac[2] < 0.56


def vs_flags(sd, dr):
    return (oracle.F_SUDDEN_DEATH if sd else 0) | (oracle.F_DISK_REWARD if dr else 0)


@pytest.mark.parametrize("n", [6, 8])
def test_vs_greedy_matches_reference(golden_dir, n):
    """OthelloEnv semantics (othello.py:151-200) with a greedy opponent: the
    oracle's reset_vs/step_vs replay the reference's recorded games."""
    v = np.load(os.path.join(golden_dir, "vs_greedy.npz"))
    combos = v["N%d_combos" % n]
    W = oracle.nwords(n)
    starts = 0
    for ci, (prot, sd, dr) in enumerate(combos):
        sel = v["N%d_combo" % n] == ci
        for g in np.unique(v["N%d_game" % n][sel]):
            idx = np.flatnonzero(sel & (v["N%d_game" % n] == g))
            s = oracle.reset_vs(n, 1, vs_flags(sd, dr), 1, 0, prot=[prot])
            assert list(s.boards[0, :W]) == list(v["N%d_start_black" % n][starts])
            assert list(s.boards[0, W:]) == list(v["N%d_start_white" % n][starts])
            starts += 1
            for k, i in enumerate(idx):
                r, d, plies = oracle.step_vs(s, vs_flags(sd, dr), 1, k + 1, [v["N%d_action" % n][i]], prot=[prot])
                assert r[0] == v["N%d_reward" % n][i] and bool(d[0]) == bool(v["N%d_done" % n][i])
                assert list(s.boards[0]) == list(v["N%d_black" % n][i]) + list(v["N%d_white" % n][i])
                assert (1 if s.meta[0] & 1 else -1) == v["N%d_turn" % n][i]
                assert plies[0] >= 1


@pytest.mark.parametrize("n,depth", [(6, 1), (6, 2), (6, 3), (8, 1), (8, 2), (8, 3), (6, 4), (6, 5), (8, 4)])
def test_maximin_matches_reference(golden_dir, n, depth):
    g = np.load(os.path.join(golden_dir, "maximin.npz" if depth <= 3 else "maximin_deep.npz"))
    k = "N%d_d%d_" % (n, depth)
    b, w, t, a = g[k + "black"], g[k + "white"], g[k + "turn"], g[k + "action"]
    s = oracle.State(n, len(a))
    s.boards[:] = np.concatenate([b, w], axis=1)
    s.meta[:] = oracle.meta_from(t)
    s.legal[:] = oracle.recompute_legal(s)
    np.testing.assert_array_equal(oracle.maximin(s, depth), a)
    if depth == 1:  # MaxiMin-1 == Greedy (README.md:48: identical rows)
        np.testing.assert_array_equal(oracle.greedy(s), a)


DEEPER = [(4, 6), (4, 7), (4, 8), (4, 9), (4, 10), (5, 6), (5, 7), (6, 6), (8, 6)]


@pytest.mark.parametrize("n,depth", DEEPER)
def test_maximin_deeper_matches_reference(golden_dir, n, depth):
    """Depths 6..10 (maximin_deeper.npz, late positions: the reference's search
    is exponential in the depth)."""
    g = np.load(os.path.join(golden_dir, "maximin_deeper.npz"))
    k = "N%d_d%d_" % (n, depth)
    b, w, t, a = g[k + "black"], g[k + "white"], g[k + "turn"], g[k + "action"]
    s = oracle.State(n, len(a))
    s.boards[:] = np.concatenate([b, w], axis=1)
    s.meta[:] = oracle.meta_from(t)
    s.legal[:] = oracle.recompute_legal(s)
    np.testing.assert_array_equal(oracle.maximin(s, depth), a)


def test_maximin_depth0_returns_no_move(golden_dir):
    """MaxiMinPolicy(0).get_action is None on every position (simple_policies.py:117-126);
    the drop-in answers so without a device call."""
    from gymothelloenv_amd.policies import MaxiMinPolicy
    g = np.load(os.path.join(golden_dir, "maximin_deeper.npz"))
    assert (g["N6_d0_action"] == -1).all() and len(g["N6_d0_action"]) > 0
    pol = MaxiMinPolicy(0)
    assert pol.get_action(None) is None and MaxiMinPolicy(-3).get_action(None) is None
    assert MaxiMinPolicy(11).max_search_depth == 11  # any depth, as the reference (:101-103)


@pytest.mark.parametrize("n", [6, 8])
def test_host_make_state_matches_reference(golden_dir, n):
    """The drop-in's host make_state / undo_state (gymothelloenv_amd/util.py, used
    for an obs that is not the env's current one) against the reference's
    util.make_state planes (util.py:48-85), including the legal plane left empty
    with a single possible move (util.py:55); float64 like the reference."""
    from gymothelloenv_amd.util import _make_state_host, undo_state
    o = np.load(os.path.join(golden_dir, "obs.npz"))
    obs, turn, legal = o["N%d_obs" % n].astype(np.int64), o["N%d_turn" % n], o["N%d_legal" % n]
    want = o["N%d_make_state" % n]
    singles = 0
    for i in range(len(turn)):
        moves = [a for a in range(n * n) if (int(legal[i][a // 64]) >> (a % 64)) & 1]
        singles += len(moves) == 1
        st = _make_state_host(obs[i], int(turn[i]), moves)
        assert st.dtype == np.float64 and st.shape == (4, n, n)
        np.testing.assert_array_equal(st, want[i].astype(np.float64))
        back = undo_state(st, int(turn[i]))
        np.testing.assert_array_equal(back, obs[i])
    assert singles > 0  # the >= 2 quirk is exercised


@pytest.mark.parametrize("n", [6, 8, 10])
def test_update_board_matches_reference(golden_dir, n):
    """update_board (othello.py:391-410) alone on the mover's disc, the
    opponent's disc, empty legal and empty illegal squares (edges.npz): the
    oracle's board after the call equals the reference's."""
    g = np.load(os.path.join(golden_dir, "edges.npz"))
    k = "ub_N%d_" % n
    W = oracle.nwords(n)
    a = g[k + "action"]
    s = oracle.State(n, len(a))
    s.boards[:] = np.concatenate([g[k + "black"].reshape(-1, W), g[k + "white"].reshape(-1, W)], axis=1)
    s.meta[:] = oracle.meta_from(g[k + "turn"])
    oracle.update_board(s, a)
    want = np.concatenate([g[k + "post_black"].reshape(-1, W), g[k + "post_white"].reshape(-1, W)], axis=1)
    np.testing.assert_array_equal(s.boards, want)


def test_maximin_depth10_late_matches_reference(golden_dir):
    """MaxiMinPolicy(10) and (12) on late 8x8 positions (edges.npz: 3-6 empty
    squares; maximin_late.npz: depth 10 at 7-10) -- the positions the C ABI's
    position-aware leaf budget admits on one board."""
    g = np.load(os.path.join(golden_dir, "edges.npz"))
    for depth in (10, 12):
        k = "mm_d%d_" % depth
        s = oracle.State(8, len(g[k + "action"]))
        s.boards[:] = np.concatenate([g[k + "black"], g[k + "white"]], axis=1)
        s.meta[:] = oracle.meta_from(g[k + "turn"])
        s.legal[:] = oracle.recompute_legal(s)
        np.testing.assert_array_equal(oracle.maximin(s, depth), g[k + "action"])
    late = os.path.join(golden_dir, "maximin_late.npz")
    if not os.path.exists(late):
        pytest.skip("maximin_late.npz not generated")
    z = np.load(late)
    s = oracle.State(8, len(z["mm_late_action"]))
    s.boards[:, 0], s.boards[:, 1] = z["mm_late_black"], z["mm_late_white"]
    s.meta[:] = oracle.meta_from(z["mm_late_turn"])
    s.legal[:] = oracle.recompute_legal(s)
    np.testing.assert_array_equal(oracle.maximin(s, 10), z["mm_late_action"])
