#!/usr/bin/env python3
"""Interleaved A/B timing of compile-time variants of the engine, in ONE process
(cdna_hip_programming.md §5.4 rule 24).

    python tools/ab_variants.py --build a=-DOTH_SHIFT32=0 b=-DOTH_SHIFT32=1   # here (CPU, hipcc)
    python tools/ab_variants.py --run a b [--envs 65536 --plies 50 ...]       # on the GPU box

Every variant must produce identical actions / final state (checked first).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "gymothelloenv_amd", "variants")


def build(specs, sizes=None):
    from gymothelloenv_amd import build as hb
    os.makedirs(VDIR, exist_ok=True)
    for spec in specs:
        name, _, flags = spec.partition("=")
        hb.build(force=True, extra_flags=flags.split(), out=os.path.join(VDIR, "liboth_%s.so" % name),
                 only_sizes=sizes)


def run(names, E, n, plies, launches, rounds, policy, check=True, init_rand=0):
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    # "head": the shipped library itself
    libs = {nm: (L.load() if nm == "head" else L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))) for nm in names}
    envs = {nm: VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device="cuda:0", lib=lib,
                             initial_rand_steps=init_rand)
            for nm, lib in libs.items()}
    for env in envs.values():
        env.reset()
    # correctness: identical trajectories
    ref = None
    for nm, env in envs.items():
        if not check:
            break
        a, _, _ = env.step_policy(policy, n_plies=plies)
        st = [t.clone() for t in env.get_state()]
        if ref is None:
            ref = (a.clone(), st)
        else:
            assert torch.equal(a, ref[0]), "variant %s diverges" % nm
            for x, y in zip(st, ref[1]):
                assert torch.equal(x, y), "variant %s diverges (state)" % nm
    bufs = {nm: (torch.empty(plies, E, dtype=torch.int32, device="cuda:0"),
                 torch.empty(plies, E, dtype=torch.int32, device="cuda:0"),
                 torch.empty(plies, E, dtype=torch.uint8, device="cuda:0")) for nm in names}
    times = {nm: [] for nm in names}
    for r in range(rounds + 1):
        for nm in names:
            env = envs[nm]
            a, rw, d = bufs[nm]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(launches):
                env.step_policy(policy, n_plies=plies, actions=a, rewards=rw, dones=d)
            e1.record()
            torch.cuda.synchronize()
            if r > 0:  # round 0 = warm-up
                times[nm].append(e0.elapsed_time(e1) * 1e3 / (launches * plies))  # us per ply
    res = {}
    for nm in names:
        t = times[nm]
        res[nm] = {"us_per_ply_median": statistics.median(t), "us_per_ply_min": min(t),
                   "steps_per_s_median": E / (statistics.median(t) * 1e-6)}
    print(json.dumps({"E": E, "N": n, "plies_per_launch": plies, "policy": policy, "results": res}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", nargs="*")
    ap.add_argument("--run", nargs="*")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--plies", type=int, default=50)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--policy", default="random")
    ap.add_argument("--init-rand", type=int, default=0, help="random-opening bound (initial_rand_steps)")
    ap.add_argument("--no-check", action="store_true", help="timing ablations: outputs differ by design")
    ap.add_argument("--sizes", help="--build: compile only these board sizes' units (e.g. 8), link the rest from the main build")
    a = ap.parse_args()
    if a.build:
        build(a.build, [int(x) for x in a.sizes.split(",")] if a.sizes else None)
    if a.run:
        run(a.run, a.envs, a.board_size, a.plies, a.launches, a.rounds, a.policy, check=not a.no_check,
            init_rand=a.init_rand)


if __name__ == "__main__":
    main()
