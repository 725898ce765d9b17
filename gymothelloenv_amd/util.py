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
import numpy as np
import torch


def _base(env):
    return env.env if hasattr(env, 'env') and not hasattr(env, '_vec') else env


def _make_state_host(obs, player_turn, possible_moves):
    """util.py:48-74's planes for an arbitrary obs, restated with np.where:
    the mover's (+1) and the opponent's (-1) entries split into the black and
    white planes by whose turn it is, the turn plane (0 black / 1 white), and
    the possible-moves plane -- set only when there are at least two moves
    (util.py:55), rows indexed by move // len(obs) as the reference does."""
    obs = np.asarray(obs)
    # keep: the plane of the side whose discs are +1 (opponent's -1 -> 0);
    # flip: the other side's (+1 -> 0, then -1 -> 1), values other than +-1 kept
    keep = np.where(obs == -1, 0, obs).astype(obs.dtype)
    flip = np.where(obs == 1, 0, np.where(obs == -1, 1, obs)).astype(obs.dtype)
    black_to_move = player_turn == -1
    black, white = (keep, flip) if black_to_move else (flip, keep)
    turn = np.zeros(obs.shape) if black_to_move else np.ones(obs.shape)
    moves = np.asarray(possible_moves, dtype=np.int64)
    legal = np.zeros(obs.shape)
    if moves.size >= 2:
        legal[moves // len(obs), moves % len(obs)] = 1
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
    """util.py:77-85: the mover-perspective board back from the black and
    white planes (the turn plane must match player_turn)."""
    assert int((player_turn + 1) / 2) == int(state[2][0][0])
    mine, theirs = (state[0], state[1]) if player_turn == -1 else (state[1], state[0])
    return mine - theirs
