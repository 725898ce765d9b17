#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants on the fused sample-and-step path
(oth_sample_step with caller uniforms), each variant's K plies captured once
in a HIP graph and replayed; one process, HIP events.  Variants must give
identical actions / log-probs first unless --no-check (timing ablations).

    python tools/ab_variants.py --build a= b=-DOTH_MS_MAX3=0      # here
    python tools/ab_sample_step.py a b [--envs 65536 --board-size 8 --lp]   # GPU box
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
    ap.add_argument("--plies", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--lp", action="store_true", help="also return log-probs and entropies")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    E, n, K = a.envs, a.board_size, a.plies
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    u = torch.rand(K, E, device=dev, generator=g)
    envs, graphs = {}, {}
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    ref = None
    print("torch up", file=sys.stderr, flush=True)
    for nm in a.names:
        lib = L.load() if nm == "head" else L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))
        print("variant %s loaded" % nm, file=sys.stderr, flush=True)
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device=dev, lib=lib)
        env.reset()

        def ply(env, k):
            return env.sample_step(logits, uniforms=u[k], log_probs=a.lp, entropy=a.lp, rewards=rew, dones=don)

        got = []  # eager plies from the same start: identical outputs across variants
        for k in range(K):
            act, lp, ent, _, _ = ply(env, k)
            got += [act.clone()] + ([lp.clone(), ent.clone()] if a.lp else [])
        if ref is None:
            ref = got
        elif not a.no_check:
            assert all(torch.equal(x, y) for x, y in zip(got, ref)), "variant %s differs" % nm
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k in range(K):
                ply(env, k)
        envs[nm], graphs[nm] = env, graph
        print("variant %s ready" % nm, file=sys.stderr, flush=True)
    times = {nm: [] for nm in a.names}
    for rd in range(a.rounds):
        print("round %d" % rd, file=sys.stderr, flush=True)
        for nm in a.names:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                graphs[nm].replay()
            e1.record()
            torch.cuda.synchronize()
            times[nm].append(e0.elapsed_time(e1) * 1e3 / (a.reps * K))
    print(json.dumps({"path": "sample_step graphed" + (" +lp/ent" if a.lp else ""), "E": E, "N": n,
                      "results": {nm: {"us_per_ply_median": statistics.median(t), "us_per_ply_min": min(t)}
                                  for nm, t in times.items()}}))


if __name__ == "__main__":
    main()
