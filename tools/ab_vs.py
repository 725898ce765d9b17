#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants of OthelloEnv's device turn loop
(oth_step_vs with a greedy protagonist, bench.vs_line's workload) in ONE process:
the variants must end in the same states with the same per-call plies (checked
first), then each variant's `--calls` calls are captured in a HIP graph and
replayed in turn.

    python tools/ab_variants.py --build old=-DOTH_VS1=0 new=          # here (CPU, hipcc)
    python tools/ab_vs.py old new [--envs 65536 --opponents random,greedy]   # GPU box
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
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--calls", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--opponents", default="random,greedy")
    ap.add_argument("--init-rand", type=int, default=10)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    dev = torch.device("cuda", 0)
    libs = {nm: L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm)) for nm in a.names}
    for opp in a.opponents.split(","):
        envs = {nm: VecOthelloEnv(a.envs, board_size=a.board_size, auto_reset=True, seed=11, device=dev, lib=lib,
                                  initial_rand_steps=a.init_rand) for nm, lib in libs.items()}
        prot = (torch.arange(a.envs, device=dev) % 3 == 0).to(torch.int8) * -2 + 1  # mixed colours
        ref = None
        for nm, env in envs.items():  # identical results first
            env.reset_vs(opp, protagonist=prot)
            plies = [env.step_vs(env.policy_actions("greedy"), opp, observe=False)[3] for _ in range(a.calls)]
            got = (torch.stack(plies), env.get_state(), env.counts_vs())
            if ref is None:
                ref = got
            else:
                assert torch.equal(got[0], ref[0]), "variant %s: plies differ" % nm
                for x, y in zip(got[1], ref[1]):
                    assert torch.equal(x, y), "variant %s: states differ" % nm
                assert torch.equal(got[2], ref[2]), "variant %s: W/D/L differ" % nm
        graphs = {}
        for nm, env in envs.items():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), env.graph_region():
                for _ in range(a.calls):
                    env.step_vs(env.policy_actions("greedy"), opp, observe=False)
            graphs[nm] = g
        times = {nm: [] for nm in a.names}
        for r in range(a.rounds + 1):
            for nm in a.names:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graphs[nm].replay()
                e1.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[nm].append(e0.elapsed_time(e1) * 1e3 / a.calls)
        print(json.dumps({"E": a.envs, "N": a.board_size, "opponent": opp, "init_rand": a.init_rand,
                          "results": {nm: {"us_per_call_median": statistics.median(t), "us_per_call_min": min(t)}
                                      for nm, t in times.items()}}), flush=True)
        for env in envs.values():
            env.close()


if __name__ == "__main__":
    main()
