"""ctypes wrapper around oracle/liboth_oracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference rules engine (othello_oracle.c).  Imported
by tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline leg only,
always as the checker; the product package gymothelloenv_amd never imports it.
All arrays use the exchange format documented in include/othello_mi355x.h.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboth_oracle.so")
BB_PATH = os.path.join(HERE, "libcpu_bitboard.so")

F_SUDDEN_DEATH = 1
F_DISK_REWARD = 2
F_AUTO_RESET = 4

_lib = None
_bb = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _stale(out, *srcs):
    return not os.path.exists(out) or any(os.path.getmtime(out) < os.path.getmtime(s) for s in srcs)


def lib():
    global _lib
    if _lib is None:
        if _stale(LIB_PATH, os.path.join(HERE, "othello_oracle.c")):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i32, u32, u64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
        L.oracle_nwords.argtypes = [i32]
        L.oracle_reset_batch.argtypes = [i32, i32, P, P, P]
        L.oracle_legal_batch.argtypes = [i32, i32, P, P, P]
        L.oracle_update_board_batch.argtypes = [i32, i32, P, P, P]
        L.oracle_step_batch.argtypes = [i32, u32, u64, u32, u64, i32, i32, P, P, P, P, P, P, P]
        L.oracle_step_batch.restype = i32
        L.oracle_reset_openings.argtypes = [i32, i32, u64, u32, u64, i32, P, P, P]
        L.oracle_rollout.argtypes = [i32, u32, i32, i32, u64, u32, u64, i32, i32, P, P, P, P, P, P, P]
        L.oracle_greedy_batch.argtypes = [i32, i32, P, P, P, P]
        L.oracle_recompute_legal.argtypes = [i32, i32, P, P, P]
        L.oracle_observe.argtypes = [i32, i32, P, P, P, P, P, P]
        L.oracle_count_disks_batch.argtypes = [i32, i32, P, P, P]
        L.oracle_maximin_batch.argtypes = [i32, i32, i32, P, P, P, P]
        L.oracle_reset_vs.argtypes = [i32, u32, i32, i32, u64, u32, u64, i32, P, P, P, P]
        L.oracle_step_vs.argtypes = [i32, u32, i32, i32, u64, u32, u64, i32, P, P, P, P, P, P, P, P, P]
        _lib = L
    return _lib


def bb_lib():
    """The bitboard CPU baseline (cpu_bitboard.cpp): bench.py's "best CPU" leg."""
    global _bb
    if _bb is None:
        if _stale(BB_PATH, os.path.join(HERE, "cpu_bitboard.cpp"),
                  os.path.join(HERE, "..", "gymothelloenv_amd", "csrc", "bitboard.hpp")):
            build()
        L = ctypes.CDLL(BB_PATH)
        P = ctypes.c_void_p
        L.cpu_bb_rollout.argtypes = [ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_int32, ctypes.c_int32, P, P, P, P, P, P, P]
        L.cpu_bb_rollout.restype = ctypes.c_int64
        _bb = L
    return _bb


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def nwords(n):
    return (n * n + 63) // 64


class State(object):
    """E boards in the exchange format (numpy, host)."""

    def __init__(self, n, E):
        W = nwords(n)
        self.n, self.E, self.W = n, E, W
        self.boards = np.zeros((E, 2 * W), dtype=np.uint64)
        self.meta = np.zeros(E, dtype=np.uint16)
        self.legal = np.zeros((E, W), dtype=np.uint64)

    def copy(self):
        s = State(self.n, self.E)
        s.boards[:] = self.boards
        s.meta[:] = self.meta
        s.legal[:] = self.legal
        return s


def reset(n, E):
    s = State(n, E)
    lib().oracle_reset_batch(n, E, _p(s.boards), _p(s.meta), _p(s.legal))
    return s


def reset_openings(n, E, seed, id_base, ply, initial_rand_steps):
    s = State(n, E)
    lib().oracle_reset_openings(n, E, seed, id_base, ply, initial_rand_steps,
                                _p(s.boards), _p(s.meta), _p(s.legal))
    return s


def legal(n, mover, opp):
    mover = np.ascontiguousarray(mover, dtype=np.uint64)
    opp = np.ascontiguousarray(opp, dtype=np.uint64)
    E = mover.shape[0]
    out = np.zeros((E, nwords(n)), dtype=np.uint64)
    lib().oracle_legal_batch(n, E, _p(mover), _p(opp), _p(out))
    return out


def update_board(s, actions):
    """update_board (othello.py:391-410) alone, in place on s.boards: the side to
    move flips from square actions[i] (any square of the board, occupied or not)
    and puts its disc there; meta and legal are untouched."""
    actions = np.ascontiguousarray(actions, dtype=np.int32)
    lib().oracle_update_board_batch(s.n, s.E, _p(s.boards), _p(s.meta), _p(actions))


def step(s, flags, actions, seed=0, id_base=0, ply=0, initial_rand_steps=0, wdl=None):
    """In-place step of State s; returns (rewards, dones, n_stepped_while_terminated).
    wdl: optional int64[3] accumulator {black wins, draws, white wins}."""
    actions = np.ascontiguousarray(actions, dtype=np.int32)
    rewards = np.zeros(s.E, dtype=np.int32)
    dones = np.zeros(s.E, dtype=np.uint8)
    errs = lib().oracle_step_batch(s.n, flags, seed, id_base, ply, initial_rand_steps, s.E,
                                   _p(s.boards), _p(s.meta), _p(s.legal), _p(actions), _p(rewards),
                                   _p(dones), _p(wdl))
    return rewards, dones, errs


def rollout(s, flags, policy, plies, seed=0, id_base=0, ply0=0, initial_rand_steps=0, record=True):
    """In-place rollout; returns (actions, rewards, dones [plies, E] or None, wdl int64[3])."""
    E = s.E
    acts = np.zeros((plies, E), dtype=np.int32) if record else None
    rews = np.zeros((plies, E), dtype=np.int32) if record else None
    dns = np.zeros((plies, E), dtype=np.uint8) if record else None
    wdl = np.zeros(3, dtype=np.int64)
    lib().oracle_rollout(s.n, flags, policy, initial_rand_steps, seed, id_base, ply0, E, plies,
                         _p(s.boards), _p(s.meta), _p(s.legal), _p(acts), _p(rews), _p(dns), _p(wdl))
    return acts, rews, dns, wdl


def rollout_parallel(s, flags, policy, plies, seed=0, id_base=0, ply0=0, initial_rand_steps=0, threads=None):
    """rollout() over contiguous board ranges on host threads (the ctypes call
    releases the GIL); boards are independent and keyed by global id, so the
    result equals one rollout() call.  For full-size replays (65,536 boards)."""
    import concurrent.futures
    E = s.E
    T = max(1, min(threads or len(os.sched_getaffinity(0)), 16, E))
    cuts = [E * k // T for k in range(T + 1)]
    acts = np.zeros((plies, E), dtype=np.int32)
    rews = np.zeros((plies, E), dtype=np.int32)
    dns = np.zeros((plies, E), dtype=np.uint8)
    wdls = np.zeros((T, 3), dtype=np.int64)

    def part(k):
        lo, hi = cuts[k], cuts[k + 1]
        sub = State(s.n, hi - lo)
        sub.boards[:] = s.boards[lo:hi]
        sub.meta[:] = s.meta[lo:hi]
        sub.legal[:] = s.legal[lo:hi]
        a, r, d, w = rollout(sub, flags, policy, plies, seed=seed, id_base=id_base + lo, ply0=ply0,
                             initial_rand_steps=initial_rand_steps)
        acts[:, lo:hi], rews[:, lo:hi], dns[:, lo:hi], wdls[k] = a, r, d, w
        s.boards[lo:hi], s.meta[lo:hi], s.legal[lo:hi] = sub.boards, sub.meta, sub.legal

    with concurrent.futures.ThreadPoolExecutor(T) as ex:
        list(ex.map(part, range(T)))
    return acts, rews, dns, wdls.sum(0)


def bb_rollout(s, plies, seed=0, id_base=0, ply0=0, record=True, wdl=None):
    """Random-play rollout with the bitboard CPU baseline, in place (auto-reset,
    sudden death irrelevant: random picks are legal).  Returns (actions,
    rewards, dones or None, wdl, env-steps taken)."""
    E = s.E
    acts = np.zeros((plies, E), dtype=np.int32) if record else None
    rews = np.zeros((plies, E), dtype=np.int32) if record else None
    dns = np.zeros((plies, E), dtype=np.uint8) if record else None
    wdl = np.zeros(3, dtype=np.int64) if wdl is None else wdl
    steps = bb_lib().cpu_bb_rollout(s.n, seed, id_base, ply0, E, plies, _p(s.boards), _p(s.meta), _p(s.legal),
                                    _p(acts), _p(rews), _p(dns), _p(wdl))
    return acts, rews, dns, wdl, steps


def greedy(s):
    out = np.zeros(s.E, dtype=np.int32)
    lib().oracle_greedy_batch(s.n, s.E, _p(s.boards), _p(s.meta), _p(s.legal), _p(out))
    return out


def maximin(s, depth):
    """MaxiMinPolicy(depth).get_action for every position of State s."""
    out = np.zeros(s.E, dtype=np.int32)
    lib().oracle_maximin_batch(s.n, depth, s.E, _p(s.boards), _p(s.meta), _p(s.legal), _p(out))
    return out


def recompute_legal(s):
    out = np.zeros_like(s.legal)
    lib().oracle_recompute_legal(s.n, s.E, _p(s.boards), _p(s.meta), _p(out))
    return out


def count_disks(s):
    """count_disks (othello.py:468-471) of every board: int32 (E, 2) = (white, black)."""
    out = np.zeros((s.E, 2), dtype=np.int32)
    lib().oracle_count_disks_batch(s.n, s.E, _p(s.boards), _p(s.meta), _p(out))
    return out


def observe(s):
    """(obs int8 (E,N,N), obs2 int8 (E,2,N,N), make_state float32 (E,4,N,N))."""
    n, E = s.n, s.E
    obs = np.zeros((E, n, n), dtype=np.int8)
    obs2 = np.zeros((E, 2, n, n), dtype=np.int8)
    ms = np.zeros((E, 4, n, n), dtype=np.float32)
    lib().oracle_observe(n, E, _p(s.boards), _p(s.meta), _p(s.legal), _p(obs), _p(obs2), _p(ms))
    return obs, obs2, ms


def meta_from(turn, terminated=False, winner=0, rand_left=0):
    """Pack reference-style (player_turn, terminated, winner) into the meta word."""
    m = np.asarray(turn) == 1
    m = m.astype(np.uint16)
    m |= (np.asarray(terminated).astype(np.uint16) << 1)
    w = np.asarray(winner)
    m |= (np.where(w == 1, 1, np.where(w == -1, 2, 0)).astype(np.uint16) << 2)
    m |= (np.asarray(rand_left).astype(np.uint16) << 8)
    return m.astype(np.uint16)


def reset_vs(n, E, flags, policy, call, seed=0, id_base=0, initial_rand_steps=0, prot=None):
    """OthelloEnv.reset for E boards (device semantics of oth_reset_vs)."""
    s = State(n, E)
    prot = None if prot is None else np.ascontiguousarray(prot, dtype=np.int8)
    lib().oracle_reset_vs(n, flags, policy, initial_rand_steps, seed, id_base, call, E, _p(prot),
                          _p(s.boards), _p(s.meta), _p(s.legal))
    return s


def step_vs(s, flags, policy, call, actions, seed=0, id_base=0, initial_rand_steps=0, prot=None, wdl=None):
    """OthelloEnv.step for E boards in place; returns (rewards, dones, plies)."""
    actions = np.ascontiguousarray(actions, dtype=np.int32)
    prot = None if prot is None else np.ascontiguousarray(prot, dtype=np.int8)
    rewards = np.zeros(s.E, dtype=np.int32)
    dones = np.zeros(s.E, dtype=np.uint8)
    plies = np.zeros(s.E, dtype=np.int32)
    lib().oracle_step_vs(s.n, flags, policy, initial_rand_steps, seed, id_base, call, s.E, _p(prot),
                         _p(actions), _p(s.boards), _p(s.meta), _p(s.legal), _p(rewards), _p(dones),
                         _p(plies), _p(wdl))
    return rewards, dones, plies
