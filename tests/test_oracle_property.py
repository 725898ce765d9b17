"""Property tests (hypothesis) of the oracle restatement on arbitrary
positions, the invariants of othello.py's rules that hold whatever the board:

  * possible_moves (othello.py:313-343) are empty squares of the board, and the
    scan is symmetric: transposing or rotating the position by 180 degrees
    transposes / rotates the moves (the eight directions map onto each other);
  * a legal move (update_board, :391-410) places one disc and turns k >= 1
    opponent discs, nothing else changes, the colours stay disjoint;
  * an illegal move with sudden_death_on_invalid_move ends the game (:417-424).

These pin the restatement beyond the reference's recorded fixtures, on
positions no game reaches; the device kernels are held to the oracle on the
same kind of positions in test_gpu_property.py."""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import oracle

E = 48
SETTINGS = dict(max_examples=40, deadline=None, derandomize=True, database=None,
                suppress_health_check=[HealthCheck.too_slow])
position = dict(n=st.sampled_from([4, 5, 6, 7, 8, 9, 10, 12, 16]), seed=st.integers(0, 2 ** 31 - 1),
                db=st.floats(0.0, 0.6), dw=st.floats(0.0, 0.6))


def _pack(mask, n):
    out = np.zeros((mask.shape[0], oracle.nwords(n)), dtype=np.uint64)
    for a in range(n * n):
        out[:, a // 64] |= mask[:, a].astype(np.uint64) << np.uint64(a % 64)
    return out


def _unpack(words, n):
    a = np.arange(n * n)
    return ((words[:, a // 64] >> (a % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)


def _masks(n, seed, db, dw):
    rng = np.random.RandomState(seed)
    u = rng.rand(E, n * n)
    return u < db, (u >= db) & (u < db + min(dw, 1.0 - db))


@settings(**SETTINGS)
@given(**position)
def test_legal_moves_are_empty_squares_and_symmetric(n, seed, db, dw):
    P, O = _masks(n, seed, db, dw)
    L = _unpack(oracle.legal(n, _pack(P, n), _pack(O, n)), n)
    assert not (L & (P | O)).any()

    def moved(f):
        Pm = f(P.reshape(E, n, n)).reshape(E, n * n)
        Om = f(O.reshape(E, n, n)).reshape(E, n * n)
        return _unpack(oracle.legal(n, _pack(Pm, n), _pack(Om, n)), n).reshape(E, n, n)

    Lb = L.reshape(E, n, n)
    np.testing.assert_array_equal(moved(lambda x: x.transpose(0, 2, 1)), Lb.transpose(0, 2, 1))
    np.testing.assert_array_equal(moved(lambda x: x[:, ::-1, ::-1]), Lb[:, ::-1, ::-1])


@settings(**SETTINGS)
@given(**position)
def test_legal_move_places_one_disc_and_turns_opponent_discs(n, seed, db, dw):
    B, Wt = _masks(n, seed, db, dw)
    rng = np.random.RandomState(seed ^ 0x3C3C)
    turn = np.where(rng.rand(E) < 0.5, 1, -1)
    tw = (turn == 1)[:, None]
    mover, opp = np.where(tw, Wt, B), np.where(tw, B, Wt)
    s = oracle.State(n, E)
    s.boards[:] = np.concatenate([_pack(B, n), _pack(Wt, n)], 1)
    s.meta[:] = oracle.meta_from(turn)
    s.legal[:] = oracle.legal(n, _pack(mover, n), _pack(opp, n))
    L = _unpack(s.legal, n)
    acts = np.full(E, -1, dtype=np.int32)
    for e in range(E):
        sq = np.flatnonzero(L[e])
        if len(sq):
            acts[e] = sq[rng.randint(len(sq))]
    live = acts >= 0
    oracle.step(s, oracle.F_SUDDEN_DEATH, acts)
    W = s.W
    B2, W2 = _unpack(s.boards[:, :W], n), _unpack(s.boards[:, W:], n)
    assert not (B2 & W2).any()
    mover2, opp2 = np.where(tw, W2, B2), np.where(tw, B2, W2)
    for e in np.flatnonzero(live):
        a = acts[e]
        turned = mover2[e] & opp[e]
        assert mover2[e, a] and not (mover[e] | opp[e])[a]
        assert turned.sum() >= 1
        np.testing.assert_array_equal(mover2[e], mover[e] | turned | (np.arange(n * n) == a))
        np.testing.assert_array_equal(opp2[e], opp[e] & ~turned)
    # boards without a possible move took an invalid action: sudden death ends them
    assert ((s.meta[~live] >> 1) & 1).all()
