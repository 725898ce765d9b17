"""The drop-in boundary at its edges (verdict r5, item 1), against fixtures the
reference itself wrote (tests/golden/edges.npz, maximin_late.npz; gen_golden.py
gen_edges / gen_maximin_late) and the oracle:

  * update_board (othello.py:391-410) called alone on any square -- the mover's
    disc, the opponent's disc, an empty legal or illegal square;
  * step() with values that are no int: the reference's `action not in
    self.possible_moves` (:417) -- 19.5 and "19" take the invalid path, a float
    equal to a member reaches update_board and raises IndexError (after the
    board was negated for a black mover, :395-396);
  * MaxiMinPolicy of depth 10 and 12 on one 8x8 board late in the game, which
    the position-aware leaf budget of the C ABI admits, while batches whose
    searches are truly above the budget are still refused.
"""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gymothelloenv_amd as g
    return g


def absolute(black, white, n):
    """(W,) black / white words -> board_state (N, N) int64: white +1, black -1."""
    sq = np.arange(n * n)
    bit = lambda w: (np.asarray(w, dtype=np.uint64)[sq // 64] >> (sq % 64).astype(np.uint64)) & np.uint64(1)
    return (bit(white).astype(np.int64) - bit(black).astype(np.int64)).reshape(n, n)


def squares(words, n):
    return [a for a in range(n * n) if (int(words[a // 64]) >> (a % 64)) & 1]


@pytest.mark.parametrize("n", [6, 8, 10])
def test_update_board_matches_reference(pkg, golden_dir, n):
    """update_board on every kind of square equals the reference's board after
    the call; turn and possible_moves are left as they were."""
    g = np.load(os.path.join(golden_dir, "edges.npz"))
    k = "ub_N%d_" % n
    W = oracle.nwords(n)
    env = pkg.OthelloBaseEnv(board_size=n, mute=True)
    env.reset()
    kinds = {"own": 0, "opponent": 0, "empty": 0}
    for i in range(len(g[k + "action"])):
        bl, wh = g[k + "black"][i].reshape(W), g[k + "white"][i].reshape(W)
        t, a = int(g[k + "turn"][i]), int(g[k + "action"][i])
        board = absolute(bl, wh, n)
        env.board_state = board
        env.player_turn = t
        moves = list(env.possible_moves)
        cell = board.reshape(-1)[a]
        kinds["empty" if cell == 0 else ("own" if cell == t else "opponent")] += 1
        env.update_board(a)
        want = absolute(g[k + "post_black"][i].reshape(W), g[k + "post_white"][i].reshape(W), n)
        np.testing.assert_array_equal(env.board_state, want, err_msg="%dx%d row %d square %d" % (n, n, i, a))
        assert env.player_turn == t and env.possible_moves == moves
    assert min(kinds.values()) > 30, kinds


@pytest.mark.parametrize("n", [6, 8, 10, 16])
def test_update_board_every_square_matches_oracle(pkg, n):
    """update_board on every square of positions from random play (mid-game,
    late, and a board already terminated, which the reference does not look at
    either) equals the oracle's cell-by-cell update_board."""
    import torch
    W = oracle.nwords(n)
    vec = pkg.VecOthelloEnv(4, board_size=n, auto_reset=False, seed=n, device="cuda:0")
    vec.step_policy("random", n_plies=n * n // 3, record=False)
    b1, m1, _ = [t.cpu().numpy() for t in vec.get_state()]
    vec.step_policy("random", n_plies=n * n, record=False)  # every game over by now
    b2, m2, _ = [t.cpu().numpy() for t in vec.get_state()]
    boards = np.concatenate([b1[:2], b2[:1]]).view(np.uint64)
    metas = np.concatenate([m1[:2], m2[:1]]).view(np.uint16)
    assert metas[2] & 2  # the last one is terminated
    env = pkg.OthelloBaseEnv(board_size=n, mute=True)
    env.reset()
    for p in range(len(boards)):
        t = 1 if metas[p] & 1 else -1
        for a in range(n * n):
            env.board_state = absolute(boards[p, :W], boards[p, W:], n)
            env.player_turn = t
            env.terminated = bool(metas[p] & 2)
            env.update_board(a)
            s = oracle.State(n, 1)
            s.boards[0], s.meta[0] = boards[p], metas[p]
            oracle.update_board(s, np.array([a], dtype=np.int32))
            np.testing.assert_array_equal(env.board_state, absolute(s.boards[0, :W], s.boards[0, W:], n),
                                          err_msg="%dx%d position %d square %d" % (n, n, p, a))
            assert env.terminated == bool(metas[p] & 2) and env.player_turn == t
    with pytest.raises(IndexError):
        env.update_board(n * n)
    with pytest.raises(IndexError):
        env.update_board(float(n))
    del torch


VALUE_OF = {"half": float, "float_member": float, "np_float64_member": np.float64,
            "np_float32_member": np.float32, "str_member": lambda v: str(int(v)), "float_nonmember": float}


def test_step_with_values_that_are_no_int(pkg, golden_dir):
    """step() decides validity by `in possible_moves` as the reference does: the
    outcome (reward and done, or the exception), the board, turn and
    possible_moves after the call all equal the reference's, in both
    sudden-death modes."""
    g = np.load(os.path.join(golden_dir, "edges.npz"))
    kinds = list(g["st_kinds"])
    envs = {sd: pkg.OthelloBaseEnv(board_size=8, mute=True, sudden_death_on_invalid_move=sd) for sd in (0, 1)}
    seen = set()
    for i in range(len(g["st_kind"])):
        kind, sd = kinds[int(g["st_kind"][i])], int(g["st_sudden"][i])
        value = VALUE_OF[kind](float(g["st_value"][i]))
        env = envs[sd]
        env.reset()
        env.board_state = absolute([g["st_black"][i]], [g["st_white"][i]], 8)
        env.set_player_turn(int(g["st_turn"][i]))
        assert env.possible_moves == squares([g["st_legal"][i]], 8)
        outcome = str(g["st_outcome"][i])
        what = "row %d: step(%r) of kind %s, sudden death %d" % (i, value, kind, sd)
        if outcome == "ok":
            _, r, d, _ = env.step(value)
            assert (r, int(d)) == (int(g["st_reward"][i]), int(g["st_done"][i])), what
        else:
            assert outcome == "IndexError", what
            with pytest.raises(IndexError):
                env.step(value)
        np.testing.assert_array_equal(env.board_state, absolute([g["st_post_black"][i]], [g["st_post_white"][i]], 8),
                                      err_msg=what)
        assert env.player_turn == int(g["st_post_turn"][i]), what
        assert env.possible_moves == squares([g["st_post_legal"][i]], 8), what
        seen.add((kind, outcome))
    assert ("float_member", "IndexError") in seen and ("half", "ok") in seen and ("str_member", "ok") in seen


def _late_positions(vec_cls, n, E, empties, seed):
    """E 8x8 positions from seeded device random play with exactly `empties`
    empty squares and a move for the side to move (host arrays)."""
    vec = vec_cls(8192, board_size=n, auto_reset=False, seed=seed, device="cuda:0")
    out_b, out_m, out_l = [], [], []
    for ply in range(n * n):
        b, m, lg = [t.cpu().numpy() for t in vec.get_state()]
        b, m, lg = b.view(np.uint64), m.view(np.uint16), lg.view(np.uint64)
        discs = np.bitwise_count(b).sum(axis=1)
        pick = (n * n - discs == empties) & ((m & 2) == 0) & (lg[:, 0] != 0)
        out_b.append(b[pick])
        out_m.append(m[pick])
        out_l.append(lg[pick])
        if sum(len(x) for x in out_b) >= E or not ((m & 2) == 0).any():
            break
        vec.step_policy("random", n_plies=1, record=False)
    b, m, lg = np.concatenate(out_b)[:E], np.concatenate(out_m)[:E], np.concatenate(out_l)[:E]
    assert len(b) == E, (empties, len(b))
    vec.close()
    return b, m, lg


@pytest.mark.parametrize("depth", [10, 12])
def test_maximin_deep_on_one_late_board(pkg, golden_dir, depth):
    """MaxiMinPolicy(10) and (12) on ONE 8x8 board (the drop-in) with 3-10 empty
    squares: the reference's own moves (edges.npz at 3-6 empty squares,
    maximin_late.npz at 7-10 for depth 10) and the oracle's at every count from
    3 to 10.  The position-blind estimate (64/6)^10 = 1.9e10 leaves is above the
    budget; the position-aware one (<= 10! at 10 empty squares) is not."""
    import torch
    env = pkg.OthelloBaseEnv(board_size=8, mute=True)
    env.reset()
    pol = pkg.MaxiMinPolicy(depth)
    pol.reset(env)

    def ask(bl, wh, t):
        env.set_board_state(absolute([bl], [wh], 8), perspective=1)
        env.set_player_turn(int(t))
        return pol.get_action(env.get_observation())

    g = np.load(os.path.join(golden_dir, "edges.npz"))
    k = "mm_d%d_" % depth
    for i in range(len(g[k + "action"])):
        want = int(g[k + "action"][i])
        assert ask(g[k + "black"][i][0], g[k + "white"][i][0], g[k + "turn"][i]) == (None if want < 0 else want)
    late = os.path.join(golden_dir, "maximin_late.npz")
    if depth == 10 and os.path.exists(late):
        z = np.load(late)
        for i in range(len(z["mm_late_action"])):
            assert ask(z["mm_late_black"][i], z["mm_late_white"][i], z["mm_late_turn"][i]) == \
                int(z["mm_late_action"][i]), "empty %d" % int(z["mm_late_empty"][i])
    for empties in range(3, 11):
        b, m, lg = _late_positions(pkg.VecOthelloEnv, 8, 2, empties, seed=empties)
        s = oracle.State(8, 2)
        s.boards[:], s.meta[:], s.legal[:] = b, m, lg
        want = oracle.maximin(s, depth)
        for i in range(2):
            t = 1 if m[i] & 1 else -1
            assert ask(b[i, 0], b[i, 1], t) == int(want[i]), "empty %d" % empties
    del torch


def test_maximin_budget_is_position_aware(pkg):
    """The C ABI's leaf budget bounds each board's search by its own position:
    a batch of late-game boards runs at depth 10 (and equals the oracle), one
    board in the middle game at depth 10 and 65,536 middle-game boards at depth 7
    are still refused before any launch, and the refusal names the estimate."""
    import torch
    from gymothelloenv_amd._lib import OthelloLibError
    b, m, lg = _late_positions(pkg.VecOthelloEnv, 8, 64, 9, seed=3)
    vec = pkg.VecOthelloEnv(64, board_size=8, device="cuda:0")
    vec.set_state(torch.from_numpy(b.view(np.int64)), torch.from_numpy(m.view(np.int16)),
                  torch.from_numpy(lg.view(np.int64)))
    s = oracle.State(8, 64)
    s.boards[:], s.meta[:], s.legal[:] = b, m, lg
    np.testing.assert_array_equal(vec.policy_actions("maximin10").cpu().numpy(), oracle.maximin(s, 10))
    np.testing.assert_array_equal(vec.policy_actions("maximin15").cpu().numpy(), oracle.maximin(s, 15))
    one = pkg.VecOthelloEnv(1, board_size=8, seed=1, device="cuda:0")
    one.step_policy("random", n_plies=20, record=False)  # 40 empty squares
    with pytest.raises(OthelloLibError, match="bounded by each board's empty squares"):
        one.policy_actions("maximin10")
    big = pkg.VecOthelloEnv(65536, board_size=8, auto_reset=True, seed=1, device="cuda:0")
    big.step_policy("random", n_plies=20, record=False)
    with pytest.raises(OthelloLibError, match="split the boards"):
        big.policy_actions("maximin7")
    with pytest.raises(OthelloLibError, match="split the boards"):
        big.step_policy("maximin5", n_plies=100, record=False)
    # depth <= 0 searches nothing (simple_policies.py:117-126): no move anywhere
    assert (vec.policy_actions("maximin0") == -1).all() and (vec.policy_actions("maximin-2") == -1).all()
    with pytest.raises(ValueError, match="unknown policy"):
        vec.policy_actions("maximinX")


def test_maximin_late_step_policy_and_opponent(pkg):
    """The position-aware budget on the other MaxiMin entry points: oth_step_policy
    (three plies from late positions, no auto-reset: 32 x 3 x (64/6)^10 leaves
    position-blind) and oth_step_vs (a MaxiMin-10 opponent late in the game) run
    where the position-blind estimate refused, and equal the oracle."""
    import torch
    b, m, lg = _late_positions(pkg.VecOthelloEnv, 8, 32, 8, seed=5)

    def loaded():
        v = pkg.VecOthelloEnv(32, board_size=8, device="cuda:0", auto_reset=False)
        v.set_state(torch.from_numpy(b.view(np.int64)), torch.from_numpy(m.view(np.int16)),
                    torch.from_numpy(lg.view(np.int64)))
        s = oracle.State(8, 32)
        s.boards[:], s.meta[:], s.legal[:] = b, m, lg
        return v, s

    vec, s = loaded()
    acts, rews, dns = vec.step_policy("maximin10", n_plies=3)
    flags = oracle.F_SUDDEN_DEATH
    for p in range(3):
        want = oracle.maximin(s, 10)
        live = (s.meta & 2) == 0
        np.testing.assert_array_equal(acts[p].cpu().numpy()[live], want[live])
        orw, od, _ = oracle.step(s, flags, np.where(live, want, -1).astype(np.int32))
        np.testing.assert_array_equal(rews[p].cpu().numpy()[live], orw[live])
        np.testing.assert_array_equal(dns[p].cpu().numpy()[live], od[live])
    vb, vm, _ = [t.cpu().numpy() for t in vec.get_state()]
    np.testing.assert_array_equal(vb.view(np.uint64), s.boards)
    np.testing.assert_array_equal(vm.view(np.uint16), s.meta)
    # OthelloEnv.step with a MaxiMin-10 opponent: the protagonist is the side to move
    vec, s = loaded()
    prot = np.where(m & 1, 1, -1).astype(np.int8)
    acts = oracle.greedy(s)
    call = vec.ply_counter
    _, r, d, plies = vec.step_vs(torch.from_numpy(acts).cuda(), opponent="maximin10",
                                 protagonist=torch.from_numpy(prot), observe=False)
    orw, od, opl = oracle.step_vs(s, flags, 11, call, acts, prot=prot)  # OTH_POLICY_MAXIMIN(10) = 11
    np.testing.assert_array_equal(r.cpu().numpy(), orw)
    np.testing.assert_array_equal(d.cpu().numpy(), od.astype(bool))
    np.testing.assert_array_equal(plies.cpu().numpy(), opl)
    vb, vm, _ = [t.cpu().numpy() for t in vec.get_state()]
    np.testing.assert_array_equal(vb.view(np.uint64), s.boards)
