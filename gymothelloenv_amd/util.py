"""util.make_state / util.undo_state (util.py:48-85) for the drop-in envs.

make_state(obs, env) returns the reference's (4, N, N) float64 planes
[black, white, turn, legal-if-at-least-two-moves], computed by the device
observe kernel (OTH_OBS_MAKE_STATE) for `env`'s current state.  `obs` must be
that env's current observation, as in every caller of the reference
(ppo_run_self_play.py:289, :298, ...).
"""
import numpy as np
import torch


def _base(env):
    return env.env if hasattr(env, 'env') and not hasattr(env, '_vec') else env


def make_state(obs, env):
    base = _base(env)
    cur = base.get_observation()
    if np.shape(obs) != np.shape(cur) or not np.array_equal(obs, cur):
        raise ValueError("make_state: obs is not the env's current observation")
    base._sync()
    st = base._vec.observe("make_state", torch.float64)
    return st[0].cpu().numpy()


def undo_state(state, player_turn):
    """util.py:77-85"""
    assert int((player_turn + 1) / 2) == int(state[2][0][0])
    if player_turn == -1:
        return state[0] - state[1]
    return state[1] - state[0]
