"""util.make_state / util.undo_state (util.py:48-85) for the drop-in envs.

make_state(obs, env) returns the reference's (4, N, N) float64 planes
[black, white, turn, legal-if-at-least-two-moves] from `obs`, `env.player_turn`
and `env.possible_moves`, exactly as util.py:48-74 combines them.  When `obs`
is the env's current observation (every caller in the reference:
ppo_run_self_play.py:289, :298, ...) the planes come from the device observe
kernel (OTH_OBS_MAKE_STATE); any other `obs` (a stored or earlier observation)
is converted by the same formula on the host, as the reference does, since
the planes then depend on an array the device does not hold.
"""
import copy

import numpy as np
import torch


def _base(env):
    return env.env if hasattr(env, 'env') and not hasattr(env, '_vec') else env


def _make_state_host(obs, player_turn, possible_moves):
    """util.py:48-74 on an arbitrary obs (the reference's quirks included:
    the legal plane only with >= 2 moves, size = len(obs))."""
    moves_number = np.array(possible_moves)
    size = len(obs)
    idx1 = moves_number // size
    idx2 = moves_number % size
    legal = np.zeros(obs.shape)
    if len(idx1) > 0 and len(idx2) > 1:
        legal[idx1, idx2] = 1
    black = copy.deepcopy(obs)
    white = copy.deepcopy(obs)
    if player_turn == -1:
        turn = np.zeros(obs.shape)
        black[black == -1] = 0
        white[white == 1] = 0
        white[white == -1] = 1
    else:
        turn = np.ones(obs.shape)
        black[black == 1] = 0
        black[black == -1] = 1
        white[white == -1] = 0
    return np.stack([black, white, turn, legal])


def make_state(obs, env):
    base = _base(env)
    cur = base.get_observation()
    if np.shape(obs) == np.shape(cur) and np.array_equal(obs, cur) and np.ndim(cur) == 2:
        base._sync()
        st = base._vec.observe("make_state", torch.float64)
        return st[0].cpu().numpy()
    return _make_state_host(obs, env.player_turn, env.possible_moves)


def undo_state(state, player_turn):
    """util.py:77-85"""
    assert int((player_turn + 1) / 2) == int(state[2][0][0])
    if player_turn == -1:
        return state[0] - state[1]
    return state[1] - state[0]
