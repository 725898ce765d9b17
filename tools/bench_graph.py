#!/usr/bin/env python3
"""The RL loop's single-ply path (masked sampling from fixed logits with
caller uniforms + step) eagerly vs captured once in a HIP graph and replayed:
per-ply wall time on one stream (HIP events), 65,536 8x8 boards by default.

    python tools/bench_graph.py [--envs 65536 --board-size 8 --plies 32 --reps 20]
"""
import argparse
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--plies", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--device-draws", action="store_true",
                    help="Philox sampling on the device (no caller uniforms), captured inside env.graph_region()")
    ap.add_argument("--fused", action="store_true", help="one oth_sample_step launch per ply instead of two calls")
    ap.add_argument("--lib", default=None, help="a variant build (gymothelloenv_amd/variants/liboth_<lib>.so)")
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd import _lib as L
    lib = L.load_path(os.path.join(ROOT, "gymothelloenv_amd", "variants", "liboth_%s.so" % a.lib)) if a.lib else None
    E, n, K = a.envs, a.board_size, a.plies
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    u = torch.rand(K, E, device=dev, generator=g)
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    acts = torch.empty(E, dtype=torch.int32, device=dev)

    def plies(env):
        for k in range(K):
            uk = None if a.device_draws else u[k]
            if a.fused:
                env.sample_step(logits, uniforms=uk, log_probs=False, entropy=False, rewards=rew, dones=don,
                                actions=acts)
            else:
                act, _, _ = env.sample_actions(logits, uniforms=uk, log_probs=False, entropy=False)
                env.step(act, rewards=rew, dones=don, observe=False)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (a.reps * K)

    eager = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device=dev, lib=lib)
    eager.reset()
    us_eager = timed(lambda: plies(eager))
    graphed = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device=dev, lib=lib)
    graphed.reset()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph), (graphed.graph_region() if a.device_draws else contextlib.nullcontext()):
        plies(graphed)
    us_graph = timed(graph.replay)
    draws = "device Philox, graph_region" if a.device_draws else "uniforms"
    path = ("sample_step(%s) [one launch]" if a.fused else "sample_actions(%s) + step") % draws
    print(json.dumps({"path": path, "lib": a.lib, "E": E, "board_size": n, "plies_per_graph": K,
                      "us_per_ply_eager": us_eager, "us_per_ply_graph": us_graph,
                      "env_steps_per_s_eager": E / (us_eager * 1e-6), "env_steps_per_s_graph": E / (us_graph * 1e-6)}))


if __name__ == "__main__":
    main()
