#!/usr/bin/env python3
"""Interleaved A/B of the learners' fused ply with its next observation
(oth_sample_step_observe: masked sample + step + make_state f32 by default)
across builds, graphed, one process:

    python tools/ab_variants.py --sizes 8 --build ssoq=-DOTH_SSO_QUAD_MAX_E=1048576   # here
    python tools/ab_ss_obs.py head ssoq [--envs 65536 --layout make_state]             # GPU box

Each variant replays K plies captured in a HIP graph from the same start state
(median of 5 replays per round, rounds interleaved); outputs must be identical
first (actions, log-probs, rewards, observations, final state)."""
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--layout", default="make_state")
    ap.add_argument("--dtype", default="float32")
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    E, n, K = a.envs, a.board_size, a.plies
    dev = torch.device("cuda", 0)
    dt = getattr(torch, a.dtype)
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    u = torch.rand(K, E, device=dev, generator=g)
    planes = {"board": 1, "absolute": 1, "legal": 1, "board_legal": 2, "make_state": 4}[a.layout]
    shape = (E, n, n) if planes == 1 else (E, planes, n, n)
    envs, graphs, starts, ref = {}, {}, {}, None
    for nm in a.names:
        lib = L.load() if nm == "head" else L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device=dev, lib=lib)
        env.step_policy("random", n_plies=20, record=False)
        start = env.get_state()
        bufs = dict(actions=torch.empty(E, dtype=torch.int32, device=dev),
                    log_probs=torch.empty(E, dtype=torch.float32, device=dev),
                    entropy=torch.empty(E, dtype=torch.float32, device=dev),
                    rewards=torch.empty(E, dtype=torch.int32, device=dev),
                    dones=torch.empty(E, dtype=torch.uint8, device=dev))
        obs = torch.empty(shape, dtype=dt, device=dev)

        def ply(k, env=env, bufs=bufs, obs=obs):
            return env.sample_step(logits, uniforms=u[k], observe=a.layout, obs=obs, **bufs)
        got = []
        for k in range(K):
            res = ply(k)
            got += [t.clone() for t in res[:4]] + [res[5].clone()]
        got += [t.clone() for t in env.get_state()] + [env.counts().clone()]
        if ref is None:
            ref = got
        else:
            assert all(torch.equal(x, y) for x, y in zip(got, ref)), "variant %s differs" % nm
        env.set_state(*start)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for k in range(K):
                ply(k)
        envs[nm], graphs[nm], starts[nm] = env, gr, start
    times = {nm: [] for nm in a.names}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds + 1):
        for nm in a.names:
            reps = []
            for _ in range(5):
                envs[nm].set_state(*starts[nm])
                torch.cuda.synchronize()
                e0.record()
                graphs[nm].replay()
                e1.record()
                torch.cuda.synchronize()
                reps.append(e0.elapsed_time(e1) * 1e3 / K)
            if r > 0:
                times[nm].append(statistics.median(reps))
    print(json.dumps({"path": "sample_step_observe %s %s graphed" % (a.layout, a.dtype), "E": E, "N": n,
                      "results": {nm: {"us_per_ply_median": statistics.median(t), "us_per_ply_min": min(t)}
                                  for nm, t in times.items()}}))


if __name__ == "__main__":
    main()
