#!/usr/bin/env python3
"""Interleaved A/B of oth_step_observe's lane layouts (k_ply_step_obs<N, LPB, BPW>,
compile-time OTH_SO_LPB / OTH_SO_BPW) against the two-launch form (oth_step +
oth_observe) and the parts alone, in ONE process, at 65,536 boards:

    python tools/ab_variants.py --sizes 8 --build so1x64=-DOTH_SO_BPW=64 so2x32="-DOTH_SO_LPB=2 -DOTH_SO_BPW=32"
    python tools/ab_step_obs.py [--variants so1x64 so2x32] [--envs 65536]    # on the GPU box

Each timing is a HIP graph of P launches replaying P plies of recorded random
play (all legal, auto-reset) from the same start state, median of 5 replays per
round, rounds interleaved over the variants; "torch/fill" is torch's fill_ of
the same observation tensor, the store-only floor.  Every variant's observations and
final state must equal the shipped library's (checked first)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "gymothelloenv_amd", "variants")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", default=[])
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--plies", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    E, n, P = a.envs, a.board_size, a.plies
    dev = torch.device("cuda", 0)
    libs = {"head": L.load()}
    libs.update({v: L.load_path(os.path.join(VDIR, "liboth_%s.so" % v)) for v in a.variants})
    rec = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev)
    rec.step_policy("random", n_plies=30, record=False)
    b0, m0, l0 = rec.get_state()
    acts = rec.step_policy("random", n_plies=P)[0]
    rec.close()
    forms = [("board", torch.int64), ("make_state", torch.float32)]
    envs = {k: VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev, lib=lib) for k, lib in libs.items()}
    outs = {(k, lay): torch.empty((E, n, n) if lay == "board" else (E, 4, n, n), dtype=dt, device=dev)
            for k in libs for lay, dt in forms}
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    # correctness: the same observations and state as the shipped library
    ref = None
    for k, env in envs.items():
        env.set_state(b0, m0, l0)
        got = []
        for i in range(P):
            lay, dt = forms[i % 2]
            o = env.step(acts[i], rewards=rew, dones=don, obs=outs[(k, lay)], obs_layout=lay)[0]
            got.append(o.clone())
        st = [t.clone() for t in env.get_state()]
        if ref is None:
            ref = (got, st)
        else:
            assert all(torch.equal(x, y) for x, y in zip(got, ref[0])), "variant %s: observations differ" % k
            assert all(torch.equal(x, y) for x, y in zip(st, ref[1])), "variant %s: state differs" % k
    graphs = {}
    for k, env in envs.items():
        for lay, dt in forms:
            env.set_state(b0, m0, l0)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), env.graph_region():
                for i in range(P):
                    env.step(acts[i], rewards=rew, dones=don, obs=outs[(k, lay)], obs_layout=lay)
            graphs[(k, "fused", lay)] = g
    # the two-launch form, the step alone, the observation alone (shipped library)
    env = envs["head"]
    for lay, dt in forms:
        for what in ("split", "obs_only"):
            env.set_state(b0, m0, l0)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), env.graph_region():
                for i in range(P):
                    if what == "split":
                        env.step(acts[i], rewards=rew, dones=don, observe=False)
                    env.observe(lay, dt, out=outs[("head", lay)])
            graphs[("head", what, lay)] = g
    env.set_state(b0, m0, l0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), env.graph_region():
        for i in range(P):
            env.step(acts[i], rewards=rew, dones=don, observe=False)
    graphs[("head", "step_only", "-")] = g
    # the floor: torch's own fill of the same observation tensor (a store-only kernel)
    for lay, dt in forms:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(P):
                outs[("head", lay)].fill_(1)
        graphs[("torch", "fill", lay)] = g
    times = {key: [] for key in graphs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds + 1):
        for key, g in graphs.items():
            envs.get(key[0], envs["head"]).set_state(b0, m0, l0)
            reps = []
            for _ in range(5):
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                reps.append(e0.elapsed_time(e1) * 1e3 / P)
            if r > 0:
                times[key].append(statistics.median(reps))
    res = {"%s/%s/%s" % key: {"us_per_ply_median": statistics.median(t), "us_per_ply_min": min(t)}
           for key, t in times.items()}
    print(json.dumps({"E": E, "N": n, "plies": P, "results": res}))


if __name__ == "__main__":
    main()
