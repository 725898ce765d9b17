"""The kernels' bitboard algorithms (csrc/bitboard.hpp, compiled for the host
with g++) against the oracle's cell-by-cell ray walk, on random boards of
every size -- a CPU check of the exact code the GPU runs."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "host", "bitboard_host.cpp")
LIB = os.path.join(HERE, "host", "libbitboard_host.so")
HDR = os.path.join(os.path.dirname(HERE), "gymothelloenv_amd", "csrc", "bitboard.hpp")


def build_host(lib=LIB, defines=()):
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared"] + list(defines) + ["-o", lib, SRC])
    return ctypes.CDLL(lib)


@pytest.fixture(scope="module")
def hostlib():
    L = build_host()
    P = ctypes.c_void_p
    L.host_legal.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P]
    L.host_flips.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    L.host_select.argtypes = [ctypes.c_uint64, ctypes.c_int]
    L.host_legal_fills.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    L.host_greedy_planes.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    L.host_fills_flips.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    L.host_greedy_planes_w.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    L.host_philox4.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, P]
    return L


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def random_boards(n, E, rng, density):
    W = oracle.nwords(n)
    cells = rng.choice(3, size=(E, n * n), p=[1 - density, density / 2, density / 2])
    mover = np.zeros((E, W), dtype=np.uint64)
    opp = np.zeros((E, W), dtype=np.uint64)
    for a in range(n * n):
        mover[:, a // 64] |= (cells[:, a] == 1).astype(np.uint64) << np.uint64(a % 64)
        opp[:, a // 64] |= (cells[:, a] == 2).astype(np.uint64) << np.uint64(a % 64)
    return cells, mover, opp


@pytest.mark.parametrize("n", list(range(4, 17)))
def test_legal_moves_host_build(hostlib, n):
    rng = np.random.RandomState(n)
    for density in (0.3, 0.6, 0.9):
        _, mover, opp = random_boards(n, 3000, rng, density)
        out = np.zeros_like(mover)
        assert hostlib.host_legal(n, len(mover), ptr(mover), ptr(opp), ptr(out)) == 0
        np.testing.assert_array_equal(out, oracle.legal(n, mover, opp))


@pytest.mark.parametrize("n", [4, 5, 6, 7, 8, 9, 10, 13, 16])
def test_flips_host_build(hostlib, n):
    """flips<N> from every legal square == the oracle's update_board diff."""
    rng = np.random.RandomState(50 + n)
    cells, mover, opp = random_boards(n, 1500, rng, 0.6)
    legal = oracle.legal(n, mover, opp)
    W = oracle.nwords(n)
    sq = np.full(len(mover), -1, dtype=np.int32)
    for e in range(len(mover)):
        moves = [a for a in range(n * n) if (int(legal[e, a // 64]) >> (a % 64)) & 1]
        if moves:
            sq[e] = moves[rng.randint(len(moves))]
    keep = sq >= 0
    mover, opp, sq = mover[keep], opp[keep], sq[keep]
    out = np.zeros_like(mover)
    assert hostlib.host_flips(n, len(mover), ptr(mover), ptr(opp), ptr(sq), ptr(out)) == 0
    # oracle: step the move as white (= mover) and diff the opponent's discs
    s = oracle.State(n, len(mover))
    s.boards[:] = np.concatenate([opp, mover], axis=1)   # black = opp, white = mover
    s.meta[:] = oracle.meta_from(np.ones(len(mover)))
    s.legal[:] = oracle.recompute_legal(s)
    oracle.step(s, 0, sq)
    np.testing.assert_array_equal(out, opp & ~s.boards[:, :W])


@pytest.mark.parametrize("W", [2, 3, 4])
def test_select_multiword_branch_free(hostlib, W):
    """select_bit_tab (two-word random play's pick: the word by selects on the
    prefix counts, then one select64_tab) gives every rank k of sparse and dense
    masks, empty words included."""
    f = hostlib.host_select_tab_w
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    rng = np.random.RandomState(40 + W)
    for _ in range(600):
        dens = rng.choice([0.0, 0.03, 0.15, 0.5, 0.95])
        words = np.array([int(sum(1 << i for i in range(64) if rng.rand() < dens)) for _ in range(W)], dtype=np.uint64)
        if rng.rand() < 0.3:
            words[rng.randint(W)] = 0
        bits = [64 * w + i for w in range(W) for i in range(64) if (int(words[w]) >> i) & 1]
        for k, b in enumerate(bits):
            assert f(ptr(words), W, k) == b, (W, [hex(int(x)) for x in words], k)


@pytest.mark.parametrize("variant", ["select64", "select64_tab"])
def test_select_variants_every_rank(hostlib, variant):
    """Both select forms (byte-parallel select64, and select64_tab with the bit
    inside the byte from k_play_rand's sel8 table), every rank k of dense and
    sparse (legal-mask-like) words."""
    sel = hostlib.host_select_tab if variant == "select64_tab" else hostlib.host_select
    sel.argtypes = [ctypes.c_uint64, ctypes.c_int]
    rng = np.random.RandomState(len(variant))
    words = [1, 1 << 63, (1 << 64) - 1, 0x8000000000000001, 0x0101010101010101, 0xF0]
    for _ in range(1500):
        dens = rng.choice([0.05, 0.15, 0.5, 0.9])
        x = 0
        for i in range(64):
            if rng.rand() < dens:
                x |= 1 << i
        words.append(x or (1 << int(rng.randint(64))))
    for x in words:
        bits = [i for i in range(64) if (x >> i) & 1]
        for k, b in enumerate(bits):
            assert sel(x, k) == b, (hex(x), k)


RAY_DIRS = [(0, 1), (1, 0), (1, 1), (1, -1), (0, -1), (-1, 0), (-1, -1), (-1, 1)]  # E S SE SW W N NW NE


@pytest.mark.parametrize("n", [4, 5, 6, 7, 8])
def test_dword_scan_and_fills_host_build(hostlib, n):
    """OneWord<N>::legal (the fills engine's dword-pair scan) == the oracle's
    legal moves; and the fills carry update_board: from every legal square the
    discs flipped (flips<N>) are exactly the contiguous run of each ray inside
    that ray direction's fill."""
    rng = np.random.RandomState(100 + n)
    for density in (0.3, 0.6, 0.9):
        _, mover, opp = random_boards(n, 1500, rng, density)
        out = np.zeros_like(mover)
        fills = np.zeros((len(mover), 8), dtype=np.uint64)
        assert hostlib.host_legal_fills(n, len(mover), ptr(mover), ptr(opp), ptr(out), ptr(fills)) == 0
        np.testing.assert_array_equal(out, oracle.legal(n, mover, opp))
        for e in range(0, len(mover), 5):
            lg = int(out[e, 0])
            for a in (b for b in range(n * n) if (lg >> b) & 1):
                f = np.zeros((1, 1), dtype=np.uint64)
                hostlib.host_flips(n, 1, ptr(mover[e:e + 1].copy()), ptr(opp[e:e + 1].copy()),
                                   ptr(np.array([a], dtype=np.int32)), ptr(f))
                runs = 0
                for d, (dr, dc) in enumerate(RAY_DIRS):
                    r, c = divmod(a, n)
                    r, c = r + dr, c + dc
                    while 0 <= r < n and 0 <= c < n and (int(fills[e, d]) >> (r * n + c)) & 1:
                        runs |= 1 << (r * n + c)
                        r, c = r + dr, c + dc
                assert runs == int(f[0, 0]), (n, e, a)


@pytest.mark.parametrize("n", [4, 5, 6, 7, 8])
def test_greedy_planes_host_build(hostlib, n):
    """OneWord<N>::greedy (every square's flip count on bit planes) plays the
    oracle's GreedyPolicy move (one simulated step per candidate,
    simple_policies.py:69-92), incl. the lowest-square tie-break and -1 when
    the mover has no move."""
    rng = np.random.RandomState(200 + n)
    for density in (0.3, 0.6, 0.85, 0.97):
        _, mover, opp = random_boards(n, 3000, rng, density)
        s = oracle.State(n, len(mover))
        s.boards[:] = np.concatenate([mover, opp], axis=1)  # black = mover, black to move
        s.meta[:] = oracle.meta_from(-np.ones(len(mover)))
        s.legal[:] = oracle.recompute_legal(s)
        out = np.zeros(len(mover), dtype=np.int32)
        assert hostlib.host_greedy_planes(n, len(mover), ptr(mover), ptr(opp), ptr(s.legal), ptr(out)) == 0
        np.testing.assert_array_equal(out, oracle.greedy(s))


def test_select_and_philox(hostlib):
    rng = np.random.RandomState(0)
    for _ in range(2000):
        x = int(rng.randint(1, 2 ** 62, dtype=np.int64)) | (int(rng.randint(0, 2)) << 63)
        bits = [i for i in range(64) if (x >> i) & 1]
        k = int(rng.randint(len(bits)))
        assert hostlib.host_select(x, k) == bits[k]
    # Philox4x32-10 known-answer vector (Random123 kat_vectors: ctr 0, key 0)
    out = np.zeros(4, dtype=np.uint32)
    hostlib.host_philox4(0, 0, 0, 0, ptr(out))
    assert [hex(v) for v in out] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]


@pytest.mark.parametrize("n", [4, 6, 8, 9, 10, 11, 12, 14, 16])
def test_multiword_fills_engine_host_build(hostlib, n):
    """legal_moves_fills == legal_moves (the oracle's legal moves) and, from
    every legal square, flips_fills (ray tables + the scan's fills, no capping
    test) == flips<N> (Kogge-Stone runs with the capping test) -- the FillsW
    engine's two halves, for one- and multi-word boards."""
    rng = np.random.RandomState(300 + n)
    W = oracle.nwords(n)
    for density in (0.3, 0.6, 0.9):
        E = 300
        _, mover, opp = random_boards(n, E, rng, density)
        legal = np.zeros_like(mover)
        out = np.zeros((E, n * n, W), dtype=np.uint64)
        assert hostlib.host_fills_flips(n, E, ptr(mover), ptr(opp), ptr(legal), ptr(out)) == 0
        np.testing.assert_array_equal(legal, oracle.legal(n, mover, opp))
        es, sqs = [], []
        for e in range(E):
            for a in range(n * n):
                if (int(legal[e, a // 64]) >> (a % 64)) & 1:
                    es.append(e)
                    sqs.append(a)
        want = np.zeros((len(es), W), dtype=np.uint64)
        assert hostlib.host_flips(n, len(es), ptr(mover[es].copy()), ptr(opp[es].copy()),
                                  ptr(np.array(sqs, dtype=np.int32)), ptr(want)) == 0
        np.testing.assert_array_equal(out[es, sqs], want)


@pytest.mark.parametrize("n", [4, 6, 8, 9, 10, 11, 12, 13, 14, 16])
def test_greedy_planes_multiword_host_build(hostlib, n):
    """PlanesW<N>::greedy (GreedyPolicy on bit planes for any W, from the
    fills of legal_moves_fills) plays the oracle's GreedyPolicy move
    (simple_policies.py:69-92), incl. the lowest-square tie-break and -1
    without a move."""
    rng = np.random.RandomState(400 + n)
    for density in (0.3, 0.6, 0.85, 0.97):
        _, mover, opp = random_boards(n, 1500, rng, density)
        s = oracle.State(n, len(mover))
        s.boards[:] = np.concatenate([mover, opp], axis=1)  # black = mover, black to move
        s.meta[:] = oracle.meta_from(-np.ones(len(mover)))
        s.legal[:] = oracle.recompute_legal(s)
        out = np.zeros(2 * len(mover), dtype=np.int32)  # [greedy move | its flip count]
        assert hostlib.host_greedy_planes_w(n, len(mover), ptr(mover), ptr(opp), ptr(s.legal), ptr(out)) == 0
        g = oracle.greedy(s)
        np.testing.assert_array_equal(out[:len(mover)], g)
        # max_flips (MaxiMin's last level): the greedy move's flip count, 0 without a move
        has = g >= 0
        f = np.zeros((int(has.sum()), oracle.nwords(n)), dtype=np.uint64)
        assert hostlib.host_flips(n, int(has.sum()), ptr(mover[has].copy()), ptr(opp[has].copy()),
                                  ptr(g[has].astype(np.int32)), ptr(f)) == 0
        cnt = np.array([sum(bin(int(w)).count("1") for w in row) for row in f], dtype=np.int32)
        np.testing.assert_array_equal(out[len(mover):][has], cnt)
        assert (out[len(mover):][~has] == 0).all()
