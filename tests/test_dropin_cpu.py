"""Host logic of the drop-in classes that needs no GPU: which action values
name a square (OthelloBaseEnv.step's membership test, othello.py:417) and the
MaxiMin depth parsing of VecOthelloEnv.policy_actions."""
import numpy as np
import pytest


def test_square_of_an_action():
    """An action is a square when it is an integer -- int, bool, numpy integer,
    a 0-d integer tensor (anything with __index__) -- and is compared with
    possible_moves by == otherwise, as `action in self.possible_moves` does."""
    import torch

    from gymothelloenv_amd.othello import _square
    for v, want in ((19, 19), (np.int64(19), 19), (np.int32(-3), -3), (True, 1), (False, 0),
                    (torch.tensor(7), 7), (2 ** 40, 2 ** 40)):
        assert _square(v) == want, v
    for v in (19.0, 19.5, np.float64(19), np.float32(19), "19", None, torch.tensor(7.0), [19]):
        assert _square(v) is None, v
    # the membership the reference computes for these (othello.py:417)
    moves = [19, 26, 37, 44]
    assert 19.0 in moves and np.float64(19) in moves and 19.5 not in moves and "19" not in moves


def test_maximin_depth_parsing_without_a_device():
    """policy_actions('maximin<d>') for d <= 0 returns no move for every board
    (the reference's search stops at the root, simple_policies.py:117-126) and
    an unparsable suffix raises ValueError -- both before any device call."""
    from gymothelloenv_amd.vec_env import VecOthelloEnv

    class Probe(VecOthelloEnv):  # no handle: only the host-side parsing runs
        def __init__(self):
            self.num_envs, self.board_size = 3, 8
            self.device = "cpu"

    import torch
    p = Probe()
    assert torch.equal(p.policy_actions("maximin0"), torch.full((3,), -1, dtype=torch.int32))
    assert torch.equal(p.policy_actions("maximin-4"), torch.full((3,), -1, dtype=torch.int32))
    with pytest.raises(ValueError, match="unknown policy"):
        p.policy_actions("maximinX")
    with pytest.raises(ValueError, match="unknown policy"):
        p.policy_actions("minimax3")
