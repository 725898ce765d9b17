"""The drop-in classes (OthelloBaseEnv / SimpleOthelloEnv / OthelloEnv and the
policies) reproduce the reference's seeded games exactly, on the GPU engine."""
import contextlib
import io
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gymothelloenv_amd as g
    return g


def enc(obs):
    return "".join("-0+"[int(v) + 1] for v in np.asarray(obs).ravel())


def test_wrapper_traces_match_reference(pkg, golden_dir):
    """Config 1: OthelloEnv / SimpleOthelloEnv driven by seeded RandomPolicy."""
    traces = json.load(open(os.path.join(golden_dir, "wrappers.json")))
    for tr in traces:
        kw = dict(tr["kw"])
        if tr["cls"] == "OthelloEnv":
            opp = pkg.RandomPolicy(seed=1)
            env = pkg.OthelloEnv(white_policy=opp, black_policy=opp, protagonist=tr["protagonist"], **kw)
        else:
            env = pkg.SimpleOthelloEnv(**kw)
        me = pkg.RandomPolicy(seed=0)
        with contextlib.redirect_stdout(io.StringIO()):
            for game in tr["games"]:
                obs = env.reset()
                me.reset(env)
                assert enc(obs) == game[0]["obs"]
                assert env.player_turn == game[0]["turn"]
                assert list(env.possible_moves) == game[0]["moves"]
                for st in game[1:]:
                    a = int(me.get_action(obs))
                    assert a == st["action"]
                    obs, r, done, info = env.step(a)
                    assert info is None
                    assert obs.dtype == np.int64
                    assert enc(obs) == st["obs"], (tr["cls"], tr["kw"])
                    assert r == st["reward"] and done == st["done"]
                    assert env.player_turn == st["turn"]
                    assert list(env.possible_moves) == st["moves"]


def test_base_env_api(pkg):
    env = pkg.OthelloBaseEnv(board_size=8, mute=True)
    assert env.possible_moves == []  # othello.py:242 until reset
    obs = env.reset()
    assert obs.shape == (8, 8) and obs.dtype == np.int64
    assert env.possible_moves == [19, 26, 37, 44] and env.player_turn == -1
    assert env.get_possible_actions() == [19, 26, 37, 44]
    assert env.count_disks() == (2, 2)
    assert env.action_space.n == 64
    obs, r, done, info = env.step(19)
    assert (r, done, info) == (0, False, None) and env.player_turn == 1
    assert env.count_disks() == (1, 4)
    assert env.board_state[2][3] == -1 and env.board_state[3][3] == -1
    # get_possible_actions(board) on an explicit canonical board (mover = +1)
    b = np.zeros((8, 8), dtype=int)
    b[0][0], b[0][1] = 1, -1
    assert env.get_possible_actions(b) == [2]
    # invalid move under sudden death: loss, stale possible_moves, turn kept
    moves = list(env.possible_moves)
    obs, r, done, _ = env.step(63)
    assert done and r == -1 and env.winner == -1 and env.player_turn == 1
    assert env.possible_moves == moves
    with pytest.raises(ValueError):
        env.step(0)
    env2 = pkg.OthelloBaseEnv(board_size=2, mute=True)
    assert env2.board_size == 4


def test_possible_actions_in_obs_and_disk_reward(pkg):
    env = pkg.OthelloBaseEnv(board_size=6, num_disk_as_reward=True, possible_actions_in_obs=True,
                             sudden_death_on_invalid_move=False, mute=True)
    obs = env.reset()
    assert obs.shape == (2, 6, 6) and obs.dtype == np.int64
    assert sorted(np.flatnonzero(obs[1].ravel()).tolist()) == env.possible_moves
    # invalid move without sudden death = pass (board unchanged, turn flips)
    before = env.board_state.copy()
    obs, r, done, _ = env.step(0)
    assert not done and r == 0 and env.player_turn == 1
    assert np.array_equal(before, env.board_state)


def reference_style_greedy(env):
    """The algorithm of simple_policies.GreedyPolicy (simple_policies.py:69-92)
    expressed against the env API, as that caller drives it: a fresh copy per
    candidate via env.__class__(board_size=, sudden_death_on_invalid_move=, mute=),
    reset / set_board_state / set_player_turn / step / count_disks."""
    me = env.player_turn
    obs = env.get_observation()
    new_env = env.__class__(board_size=env.board_size,
                            sudden_death_on_invalid_move=env.sudden_death_on_invalid_move, mute=True)
    new_env.reset()
    counts = []
    for move in env.possible_moves:
        new_env.reset()
        new_env.set_board_state(board_state=obs, perspective=me)
        new_env.set_player_turn(me)
        assert move in new_env.possible_moves
        new_env.step(move)
        w, b = new_env.count_disks()
        counts.append(w if me == 1 else b)
    new_env.close()
    return env.possible_moves[int(np.argmax(counts))]


@pytest.mark.parametrize("n", [6, 8])
def test_greedy_policy_and_make_state(pkg, golden_dir, n):
    g = np.load(os.path.join(golden_dir, "greedy.npz"))
    o = np.load(os.path.join(golden_dir, "obs.npz"))
    env = pkg.OthelloBaseEnv(board_size=n, mute=True)
    env.reset()
    pol = pkg.GreedyPolicy()
    pol.reset(env)
    for i in range(0, len(g["N%d_action" % n]), 7):
        bl, wh, t = g["N%d_black" % n][i], g["N%d_white" % n][i], int(g["N%d_turn" % n][i])
        board = np.zeros(n * n, dtype=np.int64)
        for a in range(n * n):
            if (int(bl[a // 64]) >> (a % 64)) & 1:
                board[a] = -1
            if (int(wh[a // 64]) >> (a % 64)) & 1:
                board[a] = 1
        env.set_board_state(board.reshape(n, n), perspective=1)
        env.set_player_turn(t)
        st = pkg.make_state(env.get_observation(), env)
        assert st.shape == (4, n, n) and st.dtype == np.float64
        a = pol.get_action(st)
        assert a == int(g["N%d_action" % n][i])
        assert reference_style_greedy(env) == a
    # make_state vs the reference's planes, incl. the single-legal-move quirk
    for i in range(0, len(o["N%d_turn" % n]), 11):
        bl, wh = o["N%d_black" % n][i], o["N%d_white" % n][i]
        board = np.zeros(n * n, dtype=np.int64)
        for a in range(n * n):
            board[a] = -1 if (int(bl[a // 64]) >> (a % 64)) & 1 else (1 if (int(wh[a // 64]) >> (a % 64)) & 1 else 0)
        env.board_state = board.reshape(n, n)
        env.player_turn = int(o["N%d_turn" % n][i])
        env.possible_moves = [a for a in range(n * n) if (int(o["N%d_legal" % n][i][a // 64]) >> (a % 64)) & 1]
        st = pkg.make_state(env.get_observation(), env)
        np.testing.assert_array_equal(st, o["N%d_make_state" % n][i].astype(np.float64))
        np.testing.assert_array_equal(pkg.undo_state(st, env.player_turn), env.get_observation())


def test_maximin_policy_dropin(pkg, golden_dir):
    env = pkg.OthelloBaseEnv(board_size=8, mute=True)
    env.reset()
    for depth in (1, 2, 3, 4):
        g = np.load(os.path.join(golden_dir, "maximin.npz" if depth <= 3 else "maximin_deep.npz"))
        pol = pkg.MaxiMinPolicy(depth)
        pol.reset(env)
        k = "N8_d%d_" % depth
        for i in range(0, len(g[k + "action"]), 5):
            bl, wh = g[k + "black"][i], g[k + "white"][i]
            board = np.zeros(64, dtype=np.int64)
            for a in range(64):
                board[a] = -1 if (int(bl[0]) >> a) & 1 else (1 if (int(wh[0]) >> a) & 1 else 0)
            env.set_board_state(board.reshape(8, 8), perspective=1)
            env.set_player_turn(int(g[k + "turn"][i]))
            assert pol.get_action(env.get_observation()) == int(g[k + "action"][i])
