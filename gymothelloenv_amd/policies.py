"""Scripted policies with the reference's protocol (simple_policies.py).

`reset(env)` (unwrapping `env.env` like simple_policies.py:28-32),
`get_action(obs)`, `get_test_action(obs)`, optional `seed(seed)`.

RandomPolicy draws exactly like simple_policies.py:37-41 (np.random.RandomState
index into possible_moves), so seeded games match the reference move for move.
GreedyPolicy and MaxiMinPolicy ask the device kernels (oth_policy_actions) for
the move of simple_policies.py:69-92 / :98-163 -- greedy: the move flipping the
most discs, lowest square on ties; maximin: the depth-limited max-min search
with the reference's pass handling -- instead of simulating every candidate on
copied envs.
"""
import numpy as np

from . import _lib as L
from .othello import WHITE_DISK

PROTAGONIST_TURN = 1  # simple_policies.py:8-9
OPPONENT_TURN = -1


def _base(env):
    return env.env if hasattr(env, 'env') else env


class RandomPolicy(object):
    """simple_policies.py:21-44"""

    def __init__(self, seed=0):
        self.rnd = np.random.RandomState(seed=seed)
        self.env = None

    def reset(self, env):
        self.env = _base(env)

    def seed(self, seed):
        self.rnd = np.random.RandomState(seed=seed)

    def get_action(self, obs):
        possible_moves = self.env.possible_moves
        ix = self.rnd.randint(0, len(possible_moves))
        return possible_moves[ix]

    def get_test_action(self, obs):
        return self.get_action(obs)


class GreedyPolicy(object):
    """simple_policies.py:57-95: the move the device computed for the side to move
    (the bit-plane flip counts of every square, lowest square on ties) -- read
    from the board's record, which the launch of the last step / reset wrote
    (oth_step_sync): no device call of its own."""

    def __init__(self):
        self.env = None

    def reset(self, env):
        self.env = _base(env)
        self.env._greedy_bit = L.OTH_RECORD_GREEDY  # the env's records carry the greedy move from now on

    def get_action(self, obs):
        obs = np.asarray(obs)
        if obs.ndim == 3 and obs.shape[0] == 4:  # make_state obs: same turn check as undo_state
            assert int((self.env.player_turn + 1) / 2) == int(obs[2][0][0])
        a = self.env._greedy_move()
        if a < 0:
            raise ValueError('no possible moves')
        return a

    def get_test_action(self, obs):
        return self.get_action(obs)


class MaxiMinPolicy(object):
    """simple_policies.py:98-163, searched on the device.

    max_search_depth <= 0: the reference's search stops at the root (depth 0 >=
    max_search_depth, :117-126) and get_action returns None -- no device call.
    1 .. OTH_MAXIMIN_MAX_DEPTH (10): the device search -- depth 3 and deeper with
    a whole wave per board (the root's moves and their replies spread over the
    lanes, maximin_wave.hpp).  Deeper: the same search at depth = the board's
    empty squares, which it equals (every level places a disc), once the board
    has at most 10 empty squares; earlier in the game such a move raises
    (VecOthelloEnv.policy_actions).  The search is exponential in the depth: about b**depth
    leaves for b moves per position (8x8 middle games: b ~ 10), fewer late in the
    game (at most e! for e empty squares).  The C ABI refuses calls estimated
    above OTH_MAXIMIN_LEAF_BUDGET leaves (1.7e10), bounded by the board's own
    empty squares, so one 8x8 board searches depth 10 from 10 empty squares on;
    DEEP_WARN_LEAVES bounds what runs without a warning."""

    DEEP_WARN_LEAVES = 10 ** 6

    def __init__(self, max_search_depth=1):
        self.env = None
        self.max_search_depth = int(max_search_depth)

    def reset(self, env):
        self.env = _base(env)
        n = getattr(self.env, "board_size", 8)
        b = max(2, n * n // 6)  # a typical middle-game move count (8x8: ~10)
        if self.max_search_depth > 0 and b ** self.max_search_depth > self.DEEP_WARN_LEAVES:
            import warnings
            warnings.warn("MaxiMinPolicy(%d) on %dx%d boards searches up to ~%.0e leaves per middle-game move "
                          "(one wave of the GPU per board): such moves can take seconds, or be refused above the "
                          "C ABI's leaf budget; late-game moves (few empty squares) search far fewer" %
                          (self.max_search_depth, n, n, float(b ** self.max_search_depth)), RuntimeWarning)

    def get_action(self, obs):
        if self.max_search_depth <= 0:
            return None  # search(depth=0) returns (count, None) at once (:117-126)
        vec = self.env._vec
        self.env._sync()
        a = int(vec.policy_actions("maximin%d" % self.max_search_depth).cpu()[0])
        return a if a >= 0 else None  # the reference's search returns no move then (:117-126, :157-163)

    def get_test_action(self, obs):
        return self.get_action(obs)


__all__ = ['RandomPolicy', 'GreedyPolicy', 'MaxiMinPolicy', 'PROTAGONIST_TURN', 'OPPONENT_TURN', 'WHITE_DISK']
