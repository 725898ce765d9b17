#!/usr/bin/env python3
"""MaxiMinPolicy(d) for every board (oth_policy_actions) in the shipped library
(depth >= 3 on a wave per board, k_maximin_wave) against a variant where every
depth ran one lane per board (the OTH_MAXIMIN_WAVE=0 switch of commit 53fb080,
removed after this A/B: profiles/r05/b/ab_maximin.jsonl): identical moves
first, then interleaved HIP-event timings, on mid-game boards.

    git checkout 53fb080 && python tools/ab_variants.py --sizes 8 --build mmlane=-DOTH_MAXIMIN_WAVE=0
    python tools/ab_maximin.py mmlane [--envs 65536 --depths 3 4]                # GPU box
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
    ap.add_argument("variant")
    ap.add_argument("--envs", type=int, nargs="+", default=[65536, 256, 1])
    ap.add_argument("--depths", type=int, nargs="+", default=[3, 4, 5])
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    dev = torch.device("cuda", 0)
    libs = {"head": L.load(), a.variant: L.load_path(os.path.join(VDIR, "liboth_%s.so" % a.variant))}
    out = []
    for E in a.envs:
        envs = {}
        for nm, lib in libs.items():
            envs[nm] = VecOthelloEnv(E, board_size=a.board_size, auto_reset=True, seed=5, device=dev, lib=lib)
            envs[nm].step_policy("random", n_plies=25, record=False)
        for d in a.depths:
            if E * (a.board_size ** 2 / 6) ** d > 2e9:
                continue  # keep each launch of the one-lane variant short
            pol = "maximin%d" % d
            got = {nm: env.policy_actions(pol) for nm, env in envs.items()}
            assert torch.equal(got["head"], got[a.variant]), "moves differ at depth %d" % d
            times = {nm: [] for nm in envs}
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(a.rounds):
                for nm, env in envs.items():
                    torch.cuda.synchronize()
                    e0.record()
                    env.policy_actions(pol)
                    e1.record()
                    torch.cuda.synchronize()
                    times[nm].append(e0.elapsed_time(e1) * 1e3)
            rec = {"boards": E, "depth": d, "board_size": a.board_size,
                   "us": {nm: statistics.median(t) for nm, t in times.items()}}
            print(json.dumps(rec), flush=True)
            out.append(rec)


if __name__ == "__main__":
    main()
