"""The CPU baselines bench.py times: the bitboard engine (oracle/cpu_bitboard.cpp,
the kernels' rules templates compiled for the host) must play exactly the
scalar oracle's games (same Philox stream, othello.py:412-462 semantics), so
the two CPU figures measure the same work."""
import numpy as np
import pytest

from oracle import oracle


@pytest.mark.parametrize("n", list(range(4, 17)))
def test_bitboard_baseline_equals_oracle(n):
    E, plies = 256, 3 * n * n
    s1, s2 = oracle.reset(n, E), oracle.reset(n, E)
    a1, r1, d1, w1 = oracle.rollout(s1, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, 0, plies, seed=11, id_base=5)
    a2, r2, d2, w2, steps = oracle.bb_rollout(s2, plies, seed=11, id_base=5)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(d1, d2)
    np.testing.assert_array_equal(s1.boards, s2.boards)
    np.testing.assert_array_equal(s1.meta, s2.meta)
    np.testing.assert_array_equal(s1.legal, s2.legal)
    np.testing.assert_array_equal(w1, w2)
    assert steps == E * plies  # auto-reset: every ply is an env-step
    assert w1.sum() > 0


def test_bitboard_baseline_resumes_across_calls():
    """Chunked calls (as bench.py's threads make them) equal one long call."""
    n, E = 8, 128
    s1, s2 = oracle.reset(8, E), oracle.reset(8, E)
    a1 = oracle.bb_rollout(s1, 96, seed=3)[0]
    parts = [oracle.bb_rollout(s2, 16, seed=3, ply0=16 * k)[0] for k in range(6)]
    np.testing.assert_array_equal(a1, np.concatenate(parts))
    np.testing.assert_array_equal(s1.boards, s2.boards)


def test_oracle_random_action_without_moves_is_invalid():
    """A live board with an empty possible_moves (only reachable through
    set_state) takes the invalid path (-1) like the device, instead of reading
    a stale move list."""
    n, E = 8, 4
    s = oracle.reset(n, E)
    s.legal[:] = 0  # live boards, no recorded moves
    a, r, d, _ = oracle.rollout(s, oracle.F_SUDDEN_DEATH, 0, 1, seed=0)
    assert (a[0] == -1).all()
    assert (d[0] == 1).all() and (r[0] == -1).all()  # sudden death: the mover loses


def test_threaded_oracle_rollout_equals_single_call():
    """oracle.rollout_parallel (the full-size GPU replays' checker) == rollout()."""
    s1 = oracle.reset_openings(8, 999, 4, 0, 0, 6)
    s2 = s1.copy()
    r1 = oracle.rollout(s1, 5, 1, 50, seed=4, initial_rand_steps=6)
    r2 = oracle.rollout_parallel(s2, 5, 1, 50, seed=4, initial_rand_steps=6, threads=5)
    for x, y in zip(r1, r2):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(s1.boards, s2.boards)
    np.testing.assert_array_equal(s1.meta, s2.meta)
    np.testing.assert_array_equal(s1.legal, s2.legal)
