"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container (the reference tree is not on the GPU box).
It imports the reference's `othello.py`, `simple_policies.py` and `util.py`
read-only from /root/reference, with tiny stand-ins for the modules those files
import but never compute with (gym's `Env`/`spaces`, pyglet, the `ppo` and
`Rainbow` imports at the top of util.py).  No reference source is copied: the
fixtures are inputs and outputs only (bitboards, actions, rewards, flags).

Bit convention used in every fixture: square a = row * N + col
(`othello.py:392-393`), word a // 64, bit a % 64, W = ceil(N*N / 64) words per
colour.

    python tests/golden/gen_golden.py        # rewrites tests/golden/*.npz|json
    python tests/golden/gen_golden.py masked # only masked.npz (learners' policy heads)
    python tests/golden/gen_golden.py edges  # only edges.npz (the drop-in boundary's edges)
    python tests/golden/gen_golden.py maximin_late  # only maximin_late.npz (depth 10, ~8 min on 6 cores)
"""
import contextlib
import io
import json
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = os.environ.get("OTHELLO_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

SIZES = list(range(4, 17))
COMBOS = [(sd, dr) for sd in (True, False) for dr in (False, True)]  # (sudden_death, disk_reward)


def install_shims():
    """Stand-ins for modules imported (but not used for arithmetic) by the reference."""
    gym = types.ModuleType("gym")

    class Env(object):
        pass

    gym.Env = Env
    spaces = types.ModuleType("gym.spaces")

    class Discrete(object):
        def __init__(self, n):
            self.n = n

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=None):
            self.low, self.high, self.shape = low, high, np.shape(low)

    spaces.Discrete, spaces.Box = Discrete, Box
    gym.spaces = spaces
    pyglet = types.ModuleType("pyglet")
    gl = types.ModuleType("pyglet.gl")
    pyglet.gl = gl
    ppo = types.ModuleType("ppo")
    ppo.PPO = object
    rainbow = types.ModuleType("Rainbow")
    rainbow_agent = types.ModuleType("Rainbow.agent")
    rainbow_agent.Agent = object
    rainbow.agent = rainbow_agent
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "pyglet": pyglet,
                        "pyglet.gl": gl, "ppo": ppo, "Rainbow": rainbow,
                        "Rainbow.agent": rainbow_agent})
    if REF not in sys.path:
        sys.path.insert(0, REF)


def nwords(n):
    return (n * n + 63) // 64


def pack(cells, n):
    """bool (N*N,) -> (W,) uint64."""
    w = np.zeros(nwords(n), dtype=np.uint64)
    for a in np.flatnonzero(cells):
        w[a // 64] |= np.uint64(1) << np.uint64(a % 64)
    return w


def pack_moves(moves, n):
    cells = np.zeros(n * n, dtype=bool)
    cells[list(moves)] = True
    return pack(cells, n)


def board_bits(board, n):
    flat = np.asarray(board).ravel()
    return pack(flat == -1, n), pack(flat == 1, n)


def snapshot(env, n):
    b, w = board_bits(env.board_state, n)
    return b, w, int(env.player_turn), pack_moves(env.possible_moves, n)


def gen_trajectories(othello):
    """Random play (with occasional invalid actions) in all four flag combos."""
    for n in SIZES:
        games = 12 if n <= 10 else 4
        rec = {k: [] for k in ("combo", "game", "ply", "action", "black", "white",
                               "turn", "legal", "reward", "done", "winner",
                               "prev_black", "prev_white", "prev_turn", "prev_legal")}
        starts = []
        for ci, (sd, dr) in enumerate(COMBOS):
            for g in range(games):
                rnd = np.random.RandomState(1000 * n + 100 * ci + g)
                env = othello.OthelloBaseEnv(board_size=n, sudden_death_on_invalid_move=sd,
                                             num_disk_as_reward=dr, mute=True)
                env.reset()
                b, w, t, lg = snapshot(env, n)
                starts.append((ci, g, b, w, t, lg))
                ply = 0
                done = False
                p_invalid = 0.02 if sd else 0.06
                while not done:
                    if rnd.rand() < p_invalid:
                        action = int(rnd.randint(-1, n * n + 1))
                    else:
                        pm = env.possible_moves
                        action = int(pm[rnd.randint(0, len(pm))])
                    pb, pw, pt, pl = snapshot(env, n)
                    _, reward, done, info = env.step(action)
                    assert info is None
                    b, w, t, lg = snapshot(env, n)
                    for k, v in (("combo", ci), ("game", g), ("ply", ply), ("action", action),
                                 ("black", b), ("white", w), ("turn", t), ("legal", lg),
                                 ("reward", int(reward)), ("done", bool(done)),
                                 ("winner", int(env.winner)), ("prev_black", pb),
                                 ("prev_white", pw), ("prev_turn", pt), ("prev_legal", pl)):
                        rec[k].append(v)
                    ply += 1
                # stepping a terminated game must raise (othello.py:415-416)
                try:
                    env.step(0)
                    raise AssertionError("reference did not raise after termination")
                except ValueError:
                    pass
        arrays = {k: np.array(v) for k, v in rec.items()}
        for k in ("black", "white", "legal", "prev_black", "prev_white", "prev_legal"):
            arrays[k] = arrays[k].astype(np.uint64).reshape(-1, nwords(n))
        arrays["action"] = arrays["action"].astype(np.int32)
        arrays["reward"] = arrays["reward"].astype(np.int32)
        arrays["turn"] = arrays["turn"].astype(np.int8)
        arrays["prev_turn"] = arrays["prev_turn"].astype(np.int8)
        arrays["winner"] = arrays["winner"].astype(np.int8)
        arrays["combo"] = arrays["combo"].astype(np.int8)
        arrays["combos"] = np.array(COMBOS, dtype=np.int8)
        arrays["start_black"] = np.array([s[2] for s in starts], dtype=np.uint64)
        arrays["start_white"] = np.array([s[3] for s in starts], dtype=np.uint64)
        arrays["start_legal"] = np.array([s[5] for s in starts], dtype=np.uint64)
        np.savez_compressed(os.path.join(OUT, "traj_N%d.npz" % n), **arrays)
        print("traj N=%d: %d plies" % (n, len(rec["action"])))


def gen_kat(othello):
    kat = {}
    for n in SIZES:
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        env.reset()
        b, w, _, _ = snapshot(env, n)
        legal0 = list(map(int, env.possible_moves))
        env.step(legal0[0])
        kat[str(n)] = {"black": [int(x) for x in b], "white": [int(x) for x in w],
                       "black_moves": legal0, "white_moves_after_lowest": list(map(int, env.possible_moves)),
                       "action_space_n": env.action_space.n}
    # board_size is clamped to >= 4 (othello.py:230)
    kat["clamp"] = {"requested": 2, "board_size": othello.OthelloBaseEnv(board_size=2, mute=True).board_size}
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)


def gen_greedy(othello, simple_policies, util):
    """Positions from random play -> reference GreedyPolicy's choice (make_state obs)."""
    out = {}
    for n in SIZES:
        positions = 160 if n <= 8 else (60 if n <= 12 else 25)
        rnd = np.random.RandomState(7 + n)
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        pol = simple_policies.GreedyPolicy()
        pol.reset(env)
        blacks, whites, turns, acts = [], [], [], []
        while len(acts) < positions:
            env.reset()
            done = False
            while not done and len(acts) < positions:
                obs = util.make_state(env.get_observation(), env)
                if rnd.rand() < 0.35:
                    a = int(pol.get_action(obs))
                    b, w, t, _ = snapshot(env, n)
                    blacks.append(b)
                    whites.append(w)
                    turns.append(t)
                    acts.append(a)
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        out["N%d_black" % n] = np.array(blacks, dtype=np.uint64)
        out["N%d_white" % n] = np.array(whites, dtype=np.uint64)
        out["N%d_turn" % n] = np.array(turns, dtype=np.int8)
        out["N%d_action" % n] = np.array(acts, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "greedy.npz"), **out)


def gen_obs(othello, util):
    """get_observation (1- and 2-plane) and util.make_state on 6x6 / 8x8 positions."""
    out = {}
    for n in (6, 8):
        rnd = np.random.RandomState(99 + n)
        blacks, whites, turns, legals, obs1, obs2, ms, nlegal = [], [], [], [], [], [], [], []
        env = othello.OthelloBaseEnv(board_size=n, mute=True, possible_actions_in_obs=True)
        env1 = othello.OthelloBaseEnv(board_size=n, mute=True)
        for g in range(30):
            env.reset()
            done = False
            while not done:
                o2 = env.get_observation()
                env1.board_state = env.board_state.copy()
                env1.player_turn = env.player_turn
                env1.possible_moves = list(env.possible_moves)
                o1 = env1.get_observation()
                st = util.make_state(o1, env1)
                assert o1.dtype == np.int64 and o2.dtype == np.int64 and o2.shape == (2, n, n)
                assert st.dtype == np.float64 and set(np.unique(st)) <= {0.0, 1.0}
                b, w, t, lg = snapshot(env, n)
                blacks.append(b); whites.append(w); turns.append(t); legals.append(lg)
                obs1.append(o1.astype(np.int8)); obs2.append(o2.astype(np.int8))
                ms.append(st.astype(np.uint8)); nlegal.append(len(env.possible_moves))
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
            # terminal position too (stale possible_moves, turn left on the mover)
            o2 = env.get_observation()
            env1.board_state = env.board_state.copy()
            env1.player_turn = env.player_turn
            env1.possible_moves = list(env.possible_moves)
            o1 = env1.get_observation()
            st = util.make_state(o1, env1)
            b, w, t, lg = snapshot(env, n)
            blacks.append(b); whites.append(w); turns.append(t); legals.append(lg)
            obs1.append(o1.astype(np.int8)); obs2.append(o2.astype(np.int8))
            ms.append(st.astype(np.uint8)); nlegal.append(len(env.possible_moves))
        out["N%d_black" % n] = np.array(blacks, dtype=np.uint64)
        out["N%d_white" % n] = np.array(whites, dtype=np.uint64)
        out["N%d_turn" % n] = np.array(turns, dtype=np.int8)
        out["N%d_legal" % n] = np.array(legals, dtype=np.uint64)
        out["N%d_obs" % n] = np.array(obs1)
        out["N%d_obs2" % n] = np.array(obs2)
        out["N%d_make_state" % n] = np.array(ms)
        out["N%d_nlegal" % n] = np.array(nlegal, dtype=np.int32)
        print("obs N=%d: %d positions, %d with exactly one legal move" %
              (n, len(turns), int((np.array(nlegal) == 1).sum())))
    np.savez_compressed(os.path.join(OUT, "obs.npz"), **out)


def enc(obs):
    """Mover-perspective board (values -1/0/+1) as a string over '-', '0', '+'."""
    return "".join("-0+"[int(v) + 1] for v in obs.ravel())


def gen_wrappers(othello, simple_policies):
    """OthelloEnv / SimpleOthelloEnv traces driven by seeded RandomPolicy (config 1)."""
    traces = []
    quiet = io.StringIO()
    for cls_name in ("OthelloEnv", "SimpleOthelloEnv"):
        for protagonist in (1, -1):
            for init_rand in (0, 10):
                for disk in (False, True):
                    if cls_name == "SimpleOthelloEnv" and protagonist == -1:
                        continue
                    kw = dict(board_size=8, seed=0, initial_rand_steps=init_rand,
                              num_disk_as_reward=disk)
                    if cls_name == "OthelloEnv":
                        opp = simple_policies.RandomPolicy(seed=1)
                        env = othello.OthelloEnv(white_policy=opp, black_policy=opp,
                                                 protagonist=protagonist, **kw)
                    else:
                        env = othello.SimpleOthelloEnv(**kw)
                    me = simple_policies.RandomPolicy(seed=0)
                    games = []
                    with contextlib.redirect_stdout(quiet):
                        for _ in range(6):
                            obs = env.reset()
                            me.reset(env)
                            steps = [{"obs": enc(obs), "turn": int(env.player_turn),
                                      "moves": list(map(int, env.possible_moves))}]
                            done = False
                            while not done:
                                a = int(me.get_action(obs))
                                obs, r, done, info = env.step(a)
                                steps.append({"action": a, "obs": enc(obs),
                                              "reward": int(r), "done": bool(done),
                                              "turn": int(env.player_turn),
                                              "moves": list(map(int, env.possible_moves))})
                            games.append(steps)
                    traces.append({"cls": cls_name, "protagonist": protagonist, "kw": kw,
                                   "games": games})
    with open(os.path.join(OUT, "wrappers.json"), "w") as f:
        json.dump(traces, f, separators=(",", ":"))


class RawObsGreedy(object):
    """simple_policies.GreedyPolicy's algorithm (simple_policies.py:69-92) with the
    reference's own env machinery, fed the raw observation OthelloEnv passes
    (GreedyPolicy itself expects make_state planes there and cannot run inside
    OthelloEnv -- SURVEY.md §A.4)."""

    def __init__(self, othello):
        self.othello = othello
        self.env = None

    def reset(self, env):
        self.env = env.env if hasattr(env, 'env') else env

    def get_action(self, obs):
        env = self.env
        me = env.player_turn
        sim = self.othello.OthelloBaseEnv(board_size=env.board_size,
                                          sudden_death_on_invalid_move=env.sudden_death_on_invalid_move,
                                          mute=True)
        counts = []
        for move in env.possible_moves:
            sim.reset()
            sim.set_board_state(env.board_state.copy(), perspective=1)
            sim.set_player_turn(me)
            sim.step(move)
            w, b = sim.count_disks()
            counts.append(w if me == 1 else b)
        return env.possible_moves[int(np.argmax(counts))]


def gen_vs(othello):
    """OthelloEnv (othello.py:96-214) with a deterministic greedy opponent and
    seeded protagonist actions (incl. invalid ones), initial_rand_steps = 0."""
    out = {}
    quiet = io.StringIO()
    for n in (6, 8):
        rec = {k: [] for k in ("combo", "game", "ply", "action", "reward", "done", "black", "white", "turn")}
        starts = []
        ci = 0
        combos = []
        for prot in (1, -1):
            for sd in (True, False):
                for dr in (False, True):
                    combos.append((prot, sd, dr))
                    opp = RawObsGreedy(othello)
                    env = othello.OthelloEnv(white_policy=opp, black_policy=opp, protagonist=prot, board_size=n,
                                             seed=0, initial_rand_steps=0, sudden_death_on_invalid_move=sd,
                                             num_disk_as_reward=dr)
                    rnd = np.random.RandomState(500 + 10 * n + ci)
                    with contextlib.redirect_stdout(quiet):
                        for g in range(8):
                            env.reset()
                            b, w, t, _ = snapshot(env.env, n)
                            starts.append((ci, g, b, w, t))
                            done, ply = False, 0
                            while not done:
                                pm = env.possible_moves
                                if rnd.rand() < 0.03 or not pm:
                                    a = int(rnd.randint(-1, n * n + 1))
                                else:
                                    a = int(pm[rnd.randint(0, len(pm))])
                                _, r, done, _ = env.step(a)
                                b, w, t, _ = snapshot(env.env, n)
                                for k, v in (("combo", ci), ("game", g), ("ply", ply), ("action", a),
                                             ("reward", int(r)), ("done", bool(done)), ("black", b),
                                             ("white", w), ("turn", t)):
                                    rec[k].append(v)
                                ply += 1
                    ci += 1
        for k in ("black", "white"):
            rec[k] = np.array(rec[k], dtype=np.uint64).reshape(-1, nwords(n))
        out["N%d_combo" % n] = np.array(rec["combo"], dtype=np.int8)
        out["N%d_game" % n] = np.array(rec["game"], dtype=np.int16)
        out["N%d_ply" % n] = np.array(rec["ply"], dtype=np.int16)
        out["N%d_action" % n] = np.array(rec["action"], dtype=np.int32)
        out["N%d_reward" % n] = np.array(rec["reward"], dtype=np.int32)
        out["N%d_done" % n] = np.array(rec["done"], dtype=bool)
        out["N%d_black" % n] = rec["black"]
        out["N%d_white" % n] = rec["white"]
        out["N%d_turn" % n] = np.array(rec["turn"], dtype=np.int8)
        out["N%d_combos" % n] = np.array(combos, dtype=np.int8)
        out["N%d_start_black" % n] = np.array([s_[2] for s_ in starts], dtype=np.uint64)
        out["N%d_start_white" % n] = np.array([s_[3] for s_ in starts], dtype=np.uint64)
        out["N%d_start_turn" % n] = np.array([s_[4] for s_ in starts], dtype=np.int8)
        print("vs N=%d: %d protagonist steps" % (n, len(rec["action"])))
    np.savez_compressed(os.path.join(OUT, "vs_greedy.npz"), **out)


def gen_maximin(othello, simple_policies):
    """MaxiMinPolicy(depth).get_action (simple_policies.py:98-163) on positions
    from random play, depth 1..3, N = 6 and 8."""
    out = {}
    for n, counts in ((6, {1: 120, 2: 80, 3: 40}), (8, {1: 120, 2: 60, 3: 25})):
        for depth, positions in counts.items():
            rnd = np.random.RandomState(31 * n + depth)
            env = othello.OthelloBaseEnv(board_size=n, mute=True)
            pol = simple_policies.MaxiMinPolicy(depth)
            pol.reset(env)
            blacks, whites, turns, acts = [], [], [], []
            while len(acts) < positions:
                env.reset()
                done = False
                while not done and len(acts) < positions:
                    if rnd.rand() < 0.3:
                        a = pol.get_action(env.get_observation())
                        b, w, t, _ = snapshot(env, n)
                        blacks.append(b)
                        whites.append(w)
                        turns.append(t)
                        acts.append(int(a))
                    pm = env.possible_moves
                    _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
            key = "N%d_d%d_" % (n, depth)
            out[key + "black"] = np.array(blacks, dtype=np.uint64)
            out[key + "white"] = np.array(whites, dtype=np.uint64)
            out[key + "turn"] = np.array(turns, dtype=np.int8)
            out[key + "action"] = np.array(acts, dtype=np.int32)
            print("maximin N=%d depth=%d: %d positions" % (n, depth, len(acts)))
    np.savez_compressed(os.path.join(OUT, "maximin.npz"), **out)


def gen_maximin_deep(othello, simple_policies):
    """MaxiMinPolicy(depth) beyond depth 3 (simple_policies.py:98-163): depth 4
    at N = 6 and 8, depth 5 at N = 6, on positions from random play (the
    reference's search is exponential in the depth, so fewer positions)."""
    out = {}
    for n, depth, positions in ((6, 4, 40), (6, 5, 20), (8, 4, 16)):
        rnd = np.random.RandomState(97 * n + depth)
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        pol = simple_policies.MaxiMinPolicy(depth)
        pol.reset(env)
        blacks, whites, turns, acts = [], [], [], []
        while len(acts) < positions:
            env.reset()
            done = False
            while not done and len(acts) < positions:
                if rnd.rand() < 0.25:
                    a = pol.get_action(env.get_observation())
                    b, w, t, _ = snapshot(env, n)
                    blacks.append(b)
                    whites.append(w)
                    turns.append(t)
                    acts.append(int(a))
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        key = "N%d_d%d_" % (n, depth)
        out[key + "black"] = np.array(blacks, dtype=np.uint64)
        out[key + "white"] = np.array(whites, dtype=np.uint64)
        out[key + "turn"] = np.array(turns, dtype=np.int8)
        out[key + "action"] = np.array(acts, dtype=np.int32)
        print("maximin N=%d depth=%d: %d positions" % (n, depth, len(acts)), flush=True)
    np.savez_compressed(os.path.join(OUT, "maximin_deep.npz"), **out)


def gen_maximin_deeper(othello, simple_policies):
    """MaxiMinPolicy(depth) at depth 0 and 6..10 (simple_policies.py:98-163):
    depth 0 returns no move (:117-126); depths 6..10 on 4x4 boards from any
    position, 5x5 at depth 6..7 and 6x6 / 8x8 at depth 6 on positions with at
    most `max_empty` empty squares (the reference's search is exponential in
    the depth; late positions keep it to minutes)."""
    out = {}
    plan = [(4, d, 12, 16) for d in (6, 7, 8, 9, 10)] + [(5, 6, 10, 16), (5, 7, 9, 10), (6, 6, 11, 16),
                                                          (8, 6, 9, 6), (6, 0, 40, 8)]
    for n, depth, max_empty, positions in plan:
        rnd = np.random.RandomState(131 * n + depth)
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        pol = simple_policies.MaxiMinPolicy(depth)
        pol.reset(env)
        blacks, whites, turns, acts = [], [], [], []
        while len(acts) < positions:
            env.reset()
            done = False
            while not done and len(acts) < positions:
                b, w, t, _ = snapshot(env, n)
                empty = n * n - int(np.count_nonzero(env.board_state))
                if empty <= max_empty and rnd.rand() < 0.5:
                    a = pol.get_action(env.get_observation())
                    blacks.append(b)
                    whites.append(w)
                    turns.append(t)
                    acts.append(-1 if a is None else int(a))
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        key = "N%d_d%d_" % (n, depth)
        out[key + "black"] = np.array(blacks, dtype=np.uint64)
        out[key + "white"] = np.array(whites, dtype=np.uint64)
        out[key + "turn"] = np.array(turns, dtype=np.int8)
        out[key + "action"] = np.array(acts, dtype=np.int32)
        print("maximin N=%d depth=%d: %d positions" % (n, depth, len(acts)), flush=True)
    np.savez_compressed(os.path.join(OUT, "maximin_deeper.npz"), **out)


def gen_edges(othello, simple_policies):
    """The drop-in boundary's edges, from the reference itself (edges.npz):
      * update_board (othello.py:391-410) called alone on every kind of square --
        the mover's own disc, the opponent's disc, an empty legal and an empty
        illegal square -- on positions from random play, N = 6, 8, 10; the
        board after the call (turn and possible_moves are untouched);
      * step() with values that are no int (othello.py:417's `in
        possible_moves` test): a non-member float (x.5), a float / np.float64 /
        np.float32 equal to a member, a string naming a member, a float equal to
        a non-member square; the outcome ("ok" with reward and done, or the
        exception's class name) and the board, turn and possible_moves after it;
      * MaxiMinPolicy(10) and (12) on late 8x8 positions (<= 6 empty squares)."""
    out = {}
    for n in (6, 8, 10):
        rnd = np.random.RandomState(700 + n)
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        pre_b, pre_w, turns, acts, post_b, post_w = [], [], [], [], [], []
        while len(acts) < 240:
            env.reset()
            done = False
            while not done:
                if rnd.rand() < 0.35:
                    flat = np.asarray(env.board_state).ravel()
                    me = env.player_turn
                    kinds = [np.flatnonzero(flat == me), np.flatnonzero(flat == -me),
                             np.array(env.possible_moves, dtype=int),
                             np.setdiff1d(np.flatnonzero(flat == 0), env.possible_moves)]
                    for sq in kinds:
                        if len(sq) == 0:
                            continue
                        a = int(sq[rnd.randint(0, len(sq))])
                        probe = othello.OthelloBaseEnv(board_size=n, mute=True)
                        probe.reset()
                        probe.board_state = np.array(env.board_state)
                        probe.player_turn = me
                        b, w, t, _ = snapshot(probe, n)
                        probe.update_board(a)
                        pb, pw = board_bits(probe.board_state, n)
                        pre_b.append(b)
                        pre_w.append(w)
                        turns.append(t)
                        acts.append(a)
                        post_b.append(pb)
                        post_w.append(pw)
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        key = "ub_N%d_" % n
        out[key + "black"] = np.array(pre_b, dtype=np.uint64)
        out[key + "white"] = np.array(pre_w, dtype=np.uint64)
        out[key + "turn"] = np.array(turns, dtype=np.int8)
        out[key + "action"] = np.array(acts, dtype=np.int32)
        out[key + "post_black"] = np.array(post_b, dtype=np.uint64)
        out[key + "post_white"] = np.array(post_w, dtype=np.uint64)
        print("update_board N=%d: %d calls" % (n, len(acts)), flush=True)
    # step() with values that are no int, from positions of random play (8x8, both colours to move)
    kinds = ["half", "float_member", "np_float64_member", "np_float32_member", "str_member", "float_nonmember"]
    rows = {k: [] for k in ("kind", "value", "sudden", "black", "white", "turn", "legal", "outcome", "reward",
                            "done", "post_black", "post_white", "post_turn", "post_legal")}
    rnd = np.random.RandomState(811)
    for sudden in (True, False):
        for trial in range(24):
            env = othello.OthelloBaseEnv(board_size=8, mute=True, sudden_death_on_invalid_move=sudden)
            env.reset()
            for _ in range(rnd.randint(0, 30)):
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
                if done:
                    env.reset()
            pm = env.possible_moves
            member = int(pm[rnd.randint(0, len(pm))])
            empty = np.setdiff1d(np.flatnonzero(np.asarray(env.board_state).ravel() == 0), pm)
            nonmember = int(empty[rnd.randint(0, len(empty))]) if len(empty) else 64
            values = {"half": member + 0.5, "float_member": float(member),
                      "np_float64_member": np.float64(member), "np_float32_member": np.float32(member),
                      "str_member": str(member), "float_nonmember": float(nonmember)}
            for k in kinds:
                e2 = othello.OthelloBaseEnv(board_size=8, mute=True, sudden_death_on_invalid_move=sudden)
                e2.reset()
                e2.board_state = np.array(env.board_state)
                e2.set_player_turn(env.player_turn)
                b, w, t, lg = snapshot(e2, 8)
                try:
                    _, r, d, _ = e2.step(values[k])
                    outcome, r, d = "ok", int(r), int(bool(d))
                except Exception as ex:  # the reference's own exception (IndexError for a float member)
                    outcome, r, d = type(ex).__name__, 0, 0
                pb, pw, pt, plg = snapshot(e2, 8)
                for name, v in (("kind", kinds.index(k)), ("value", float(values[k])), ("sudden", int(sudden)), ("black", b[0]), ("white", w[0]),
                                ("turn", t), ("legal", lg[0]), ("outcome", outcome), ("reward", r), ("done", d),
                                ("post_black", pb[0]), ("post_white", pw[0]), ("post_turn", pt),
                                ("post_legal", plg[0])):
                    rows[name].append(v)
    for name, v in rows.items():
        dt = {"outcome": "U16", "kind": np.int8, "sudden": np.int8, "turn": np.int8, "post_turn": np.int8,
              "reward": np.int32, "done": np.int8, "value": np.float64}.get(name, np.uint64)
        out["st_" + name] = np.array(v, dtype=dt)
    out["st_kinds"] = np.array(kinds, dtype="U20")
    print("step with non-int values: %d calls, outcomes %s" % (len(rows["kind"]), sorted(set(rows["outcome"]))),
          flush=True)
    # MaxiMinPolicy(10) / (12) on late 8x8 positions
    for depth in (10, 12):
        rnd = np.random.RandomState(900 + depth)
        env = othello.OthelloBaseEnv(board_size=8, mute=True)
        pol = simple_policies.MaxiMinPolicy(depth)
        pol.reset(env)
        blacks, whites, turns, acts = [], [], [], []
        while len(acts) < 8:
            env.reset()
            done = False
            while not done and len(acts) < 8:
                empty = 64 - int(np.count_nonzero(env.board_state))
                if 3 <= empty <= 6 and rnd.rand() < 0.5:
                    a = pol.get_action(env.get_observation())
                    b, w, t, _ = snapshot(env, 8)
                    blacks.append(b)
                    whites.append(w)
                    turns.append(t)
                    acts.append(-1 if a is None else int(a))
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        key = "mm_d%d_" % depth
        out[key + "black"] = np.array(blacks, dtype=np.uint64)
        out[key + "white"] = np.array(whites, dtype=np.uint64)
        out[key + "turn"] = np.array(turns, dtype=np.int8)
        out[key + "action"] = np.array(acts, dtype=np.int32)
        print("maximin 8x8 depth=%d: %d late positions" % (depth, len(acts)), flush=True)
    np.savez_compressed(os.path.join(OUT, "edges.npz"), **out)


def _maximin_late_task(args):
    """One MaxiMinPolicy(depth) call on the 8x8 position a seeded random game
    reaches with exactly `empty` empty squares (a worker process)."""
    empty_target, depth, seed = args
    install_shims()
    import othello  # noqa: E402  (reference, read-only)
    import simple_policies  # noqa: E402
    rnd = np.random.RandomState(seed)
    while True:
        env = othello.OthelloBaseEnv(board_size=8, mute=True)
        env.reset()
        done = False
        while not done:
            empty = 64 - int(np.count_nonzero(env.board_state))
            if empty == empty_target and env.possible_moves:
                pol = simple_policies.MaxiMinPolicy(depth)
                pol.reset(env)
                a = pol.get_action(env.get_observation())
                b, w, t, _ = snapshot(env, 8)
                return int(b[0]), int(w[0]), t, -1 if a is None else int(a)
            pm = env.possible_moves
            _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))


def gen_maximin_late():
    """MaxiMinPolicy(10) on 8x8 positions with 7-10 empty squares
    (maximin_late.npz): the reference's search takes ~2 s at 7 empty squares and
    ~7 minutes at 10, so the positions run in parallel worker processes."""
    import multiprocessing
    tasks = [(e, 10, 4000 + 10 * e + k) for e in (7, 8, 9, 10) for k in range(2)]
    with multiprocessing.get_context("spawn").Pool(min(len(tasks), 6)) as pool:
        res = pool.map(_maximin_late_task, tasks, chunksize=1)
    out = {"mm_late_black": np.array([r[0] for r in res], dtype=np.uint64),
           "mm_late_white": np.array([r[1] for r in res], dtype=np.uint64),
           "mm_late_turn": np.array([r[2] for r in res], dtype=np.int8),
           "mm_late_action": np.array([r[3] for r in res], dtype=np.int32),
           "mm_late_empty": np.array([t[0] for t in tasks], dtype=np.int32),
           "mm_late_depth": np.array([t[1] for t in tasks], dtype=np.int32)}
    print("maximin 8x8 depth 10 at 7-10 empty squares: %d positions" % len(res), flush=True)
    np.savez_compressed(os.path.join(OUT, "maximin_late.npz"), **out)


def install_learner_shims():
    """Stand-ins for what the learners' modules import but the policy heads never
    use: torch.utils.tensorboard (ppo.py:7; tensorboard is absent), the
    un-vendored `baselines` behind a2c_ppo_acktr/envs.py (utils.py:7 imports only
    the VecNormalize name).  The `ppo` stub util.py needed is dropped so the real
    ppo.py is imported."""
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    envs = types.ModuleType("pytorch_a2c_ppo_acktr_gail.a2c_ppo_acktr.envs")
    envs.VecNormalize = type("VecNormalize", (object,), {})
    sys.modules.update({"torch.utils.tensorboard": tb, "pytorch_a2c_ppo_acktr_gail.a2c_ppo_acktr.envs": envs})
    sys.modules.pop("ppo", None)


def gen_masked(othello):
    """The learners' masked policy heads on fixed logits, computed by the
    reference's own code:
      * Policy.act (model.py:60-99) with deterministic=True (mode) and False
        (torch-seeded sample), actions and log-probs, through a Policy whose
        base returns the fixture logits as actor features and whose
        distributions.Categorical head has an identity linear layer;
      * Policy.evaluate_actions (model.py:156-178): per-row log-probs of given
        actions (legal, illegal and out of range) and dist_entropy (one row
        per call, so the returned mean is the row's entropy);
      * PPO.get_action (ppo.py:228-262): the renormalised probabilities over
        possible_moves and np.random.choice's draw, with the uniform u that
        numpy's legacy stream supplies to it (np.random.seed(k) then one
        random_sample()).
    Positions (possible_moves) come from reference random games; rows with no
    legal move, exactly one, and tied logits are included."""
    import torch
    import torch.nn as nn
    install_learner_shims()
    from pytorch_a2c_ppo_acktr_gail.a2c_ppo_acktr import model as M  # noqa: E402  (reference)
    from pytorch_a2c_ppo_acktr_gail.a2c_ppo_acktr.distributions import Categorical as RefCategorical  # noqa: E402
    import ppo as P  # noqa: E402  (reference)

    class Features(nn.Module):  # base(inputs, rnn_hxs, masks) -> (value, actor_features, rnn_hxs)
        def forward(self, inputs, rnn_hxs, masks):
            return torch.zeros(inputs.shape[0], 1), inputs, rnn_hxs

    out = {}
    for n in (6, 8):
        nn_sq = n * n
        rnd = np.random.RandomState(300 + n)
        env = othello.OthelloBaseEnv(board_size=n, mute=True)
        moves = []
        while len(moves) < 1500:
            env.reset()
            done = False
            while not done:
                moves.append(list(env.possible_moves))
                pm = env.possible_moves
                _, _, done, _ = env.step(int(pm[rnd.randint(0, len(pm))]))
        moves = moves[:1500] + [[] for _ in range(24)]  # + rows with no legal move
        R = len(moves)
        logits = (rnd.standard_normal((R, nn_sq)) * 3).astype(np.float32)
        logits[::17] = 1.25  # ties: the mode is the lowest legal square
        pol = M.Policy.__new__(M.Policy)
        nn.Module.__init__(pol)
        pol.base = Features()
        pol.dist = RefCategorical(nn_sq, nn_sq)
        with torch.no_grad():
            pol.dist.linear.weight.copy_(torch.eye(nn_sq))
            pol.dist.linear.bias.zero_()
        pol.i, pol.e = 1, 1
        x = torch.from_numpy(logits)
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            _, mode_a, mode_lp, _ = pol.act(x, None, None, moves, deterministic=True)
            torch.manual_seed(n)
            _, samp_a, samp_lp, _ = pol.act(x, None, None, moves, deterministic=False)
            eval_a = samp_a.clone()
            k = np.arange(R)
            eval_a[k % 5 == 1, 0] = torch.from_numpy(rnd.randint(-3, nn_sq + 3, size=int((k % 5 == 1).sum())))
            eval_lp, full_ent = [], []
            for i in range(R):
                _, lp, ent, _ = pol.evaluate_actions(x[i:i + 1], None, None, eval_a[i:i + 1], [moves[i]])
                eval_lp.append(float(lp.reshape(-1)[0]))
                full_ent.append(float(ent))
        # PPO.get_action: renormalised probabilities + np.random.choice
        agent = P.PPO.__new__(P.PPO)
        agent.env = types.SimpleNamespace(possible_moves=None)

        class Probs(object):
            def get_action_probs(self, state):
                return torch.softmax(state, dim=1)  # ActorCritic.action_and_value's softmax (ppo.py:73)

        agent.policy_old = Probs()
        seen = {}
        real_choice = np.random.choice

        def spy(a, p=None, **kw):
            seen["p"] = np.array(p, dtype=np.float64)
            return real_choice(a, p=p, **kw)

        ppo_u, ppo_a, ppo_p = np.zeros(R), np.full(R, -1, dtype=np.int32), np.zeros((R, nn_sq))
        np.random.choice = spy
        try:
            for i in range(R):
                if not moves[i]:
                    continue  # np.random.choice([]) fails in the reference (no legal move)
                agent.env.possible_moves = moves[i]
                np.random.seed(10000 + i)
                ppo_u[i] = np.random.random_sample()
                np.random.seed(10000 + i)
                ppo_a[i] = agent.get_action(logits[i])
                ppo_p[i, moves[i]] = seen["p"]
        finally:
            np.random.choice = real_choice
        legal = np.array([pack_moves(m, n) for m in moves], dtype=np.uint64)
        key = "N%d_" % n
        out.update({key + "logits": logits, key + "legal": legal,
                    key + "nlegal": np.array([len(m) for m in moves], dtype=np.int32),
                    key + "mode_action": mode_a.numpy().reshape(-1).astype(np.int32),
                    key + "mode_logp": np.asarray(mode_lp, dtype=np.float32).reshape(-1),
                    key + "sample_action": samp_a.numpy().reshape(-1).astype(np.int32),
                    key + "sample_logp": np.asarray(samp_lp, dtype=np.float32).reshape(-1),
                    key + "eval_action": eval_a.numpy().reshape(-1).astype(np.int32),
                    key + "eval_logp": np.array(eval_lp, dtype=np.float32),
                    key + "full_entropy": np.array(full_ent, dtype=np.float32),
                    key + "ppo_u": ppo_u, key + "ppo_action": ppo_a, key + "ppo_probs": ppo_p})
        print("masked N=%d: %d rows (%d without a legal move, %d with one)" %
              (n, R, sum(1 for m in moves if not m), sum(1 for m in moves if len(m) == 1)))
    np.savez_compressed(os.path.join(OUT, "masked.npz"), **out)


def main():
    install_shims()
    import othello  # noqa: E402  (reference, read-only)
    import simple_policies  # noqa: E402
    import util  # noqa: E402
    if sys.argv[1:] == ["masked"]:
        gen_masked(othello)
        return
    if sys.argv[1:] == ["maximin_deep"]:
        gen_maximin_deep(othello, simple_policies)
        return
    if sys.argv[1:] == ["maximin_deeper"]:
        gen_maximin_deeper(othello, simple_policies)
        return
    if sys.argv[1:] == ["edges"]:
        gen_edges(othello, simple_policies)
        return
    if sys.argv[1:] == ["maximin_late"]:
        gen_maximin_late()
        return
    gen_kat(othello)
    gen_trajectories(othello)
    gen_greedy(othello, simple_policies, util)
    gen_obs(othello, util)
    gen_wrappers(othello, simple_policies)
    gen_vs(othello)
    gen_maximin(othello, simple_policies)
    gen_maximin_deep(othello, simple_policies)
    gen_maximin_deeper(othello, simple_policies)
    gen_edges(othello, simple_policies)
    gen_maximin_late()
    gen_masked(othello)


if __name__ == "__main__":
    main()
