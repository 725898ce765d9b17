"""gymothelloenv_amd -- MI355X-native vectorised Othello rules engine.

Hot path of omurammm/GymOthelloEnv (othello.py's legal moves, flips,
terminal/score) as HIP kernels for gfx950 behind a C ABI
(include/othello_mi355x.h, library liboth_mi355x.so in this directory).

    VecOthelloEnv            E boards in HBM (the performance path)
    OthelloBaseEnv,          drop-in single-board classes with the
    SimpleOthelloEnv,        reference's constructor / attributes / 4-tuple step
    OthelloEnv
    RandomPolicy, GreedyPolicy, MaxiMinPolicy, make_state, undo_state
    masked_sample, masked_log_prob   policy-head sampling over legal squares
"""
from ._lib import LIB_PATH, OthelloLibError, load  # noqa: F401

BLACK_DISK, NO_DISK, WHITE_DISK = -1, 0, 1


def __getattr__(name):
    # lazy: importing the package must not touch the GPU (build() runs on CPU hosts)
    if name in ("VecOthelloEnv", "legal_moves"):
        from . import vec_env
        return getattr(vec_env, name)
    if name in ("OthelloBaseEnv", "SimpleOthelloEnv", "OthelloEnv"):
        from . import othello
        return getattr(othello, name)
    if name in ("RandomPolicy", "GreedyPolicy", "MaxiMinPolicy"):
        from . import policies
        return getattr(policies, name)
    if name in ("masked_sample", "masked_log_prob"):
        from . import masked
        return getattr(masked, name)
    if name in ("make_state", "undo_state"):
        from . import util
        return getattr(util, name)
    raise AttributeError(name)
