#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants of the single-ply kernels (ply.hpp)
in ONE process: oth_step with recorded random-play actions (k_ply_step) and
oth_step_policy(random, 1 ply) (k_ply_rand), each as P launches replayed from a
HIP graph (no host in the loop), at every board count given.  Every variant
must end in the same state as the recording (checked first).

    python tools/ab_variants.py --build a= b=-DOTH_PLY_W8=0          # here (CPU, hipcc)
    python tools/ab_ply.py a b [--envs 65536,1048576 --plies 32 --rounds 6]   # GPU box
"""
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
    ap.add_argument("names", nargs="+")
    ap.add_argument("--envs", default="65536,1048576")
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--plies", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    dev = torch.device("cuda", 0)
    libs = {nm: L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm)) for nm in a.names}
    n, P = a.board_size, a.plies
    out = {}
    for E in [int(x) for x in a.envs.split(",")]:
        envs = {nm: VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev, lib=lib)
                for nm, lib in libs.items()}
        first = envs[a.names[0]]
        first.step_policy("random", n_plies=30, record=False)
        b0, m0, l0 = [t.clone() for t in first.get_state()]
        acts = torch.empty(P, E, dtype=torch.int32, device=dev)
        first.step_policy("random", n_plies=P, actions=acts, rewards=torch.empty_like(acts),
                          dones=torch.empty(P, E, dtype=torch.uint8, device=dev))
        want = [t.clone() for t in first.get_state()]
        rew = torch.empty(E, dtype=torch.int32, device=dev)
        don = torch.empty(E, dtype=torch.uint8, device=dev)
        a1 = torch.empty(1, E, dtype=torch.int32, device=dev)
        graphs = {}
        for nm, env in envs.items():
            env.set_state(b0, m0, l0)
            env.ply_counter = 30
            g_step, g_rand = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_step), env.graph_region():
                for i in range(P):
                    env.step(acts[i], rewards=rew, dones=don, observe=False)
            with torch.cuda.graph(g_rand), env.graph_region():
                for i in range(P):
                    env.step_policy("random", n_plies=1, actions=a1, rewards=rew[None], dones=don[None])
            graphs[nm] = (g_step, g_rand)
            env.set_state(b0, m0, l0)
            g_step.replay()
            torch.cuda.synchronize()
            for x, y in zip(env.get_state(), want):
                assert torch.equal(x, y), "variant %s: replay differs from the recording" % nm
        ref_rand = None
        for nm, env in envs.items():  # the random plies: identical across variants (same graph slot counters)
            env.set_state(b0, m0, l0)
            graphs[nm][1].replay()
            torch.cuda.synchronize()
            st = [t.clone() for t in env.get_state()]
            if ref_rand is None:
                ref_rand = st
            for x, y in zip(st, ref_rand):
                assert torch.equal(x, y), "variant %s: random plies differ" % nm
        times = {nm: {"step": [], "rand": []} for nm in a.names}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(a.rounds + 1):
            for nm in a.names:
                for k, g in (("step", graphs[nm][0]), ("rand", graphs[nm][1])):
                    envs[nm].set_state(b0, m0, l0)
                    torch.cuda.synchronize()
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    if r:
                        times[nm][k].append(e0.elapsed_time(e1) * 1e3 / P)
        out[E] = {nm: {k: {"us_per_ply_median": statistics.median(v), "us_per_ply_min": min(v)}
                       for k, v in times[nm].items()} for nm in a.names}
        print(json.dumps({"E": E, "N": n, "plies": P, "results": out[E]}), flush=True)
        for env in envs.values():
            env.close()
        del graphs, envs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
