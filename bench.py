#!/usr/bin/env python3
"""Benchmark: env-steps/s of on-device random play on 65,536 8x8 boards per GPU
(BASELINE.json `metric`, config 2; N GPUs = config 4's weak-scaled shards).

A step = one ply applied to every board of the shard (one OthelloBaseEnv.step
per board, pass resolution included), the mover choosing uniformly among its
possible_moves (RandomPolicy, simple_policies.py:37-41) from a Philox stream;
finished games auto-reset.  Boards, actions, rewards and dones stay in HBM.
`--plies-per-launch P` runs P plies per kernel launch (board state kept in
registers between plies, every ply's action / reward / done still stored).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel
(k_play<8, random>) by its algorithmic HBM bytes per launch over its average
launch time (HIP events on the launch stream); `traffic` comes from the
rocprofv3 PMC summary committed under profiles/ (null if absent).
`cpu_baseline` times the oracle's scalar restatement of othello.py on the
host cores (one batch of boards per thread) over a bounded sample.
`masked_sample` is a side measurement of the learners' masked-categorical
kernel against the HBM peak.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "env-steps/sec (random policy, 65,536\u00d78\u00d78 boards) at 1/2/4/8 GPUs; HBM GB/s vs peak"


def algorithmic_bytes_per_launch(E, W, plies, record=True):
    """HBM bytes one k_play launch must move: board state in and out once
    (boards 16W + legal 8W + meta 2, each way) plus per ply the action (4),
    reward (4) and done (1) of every board."""
    state = 2 * (16 * W + 8 * W + 2)
    per_ply = (4 + 4 + 1) if record else 0
    return E * (state + plies * per_ply)


def cpu_threads():
    """Host cores this process may use: the affinity set, capped by the job's
    thread budget (OMP_NUM_THREADS is the box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_baseline(seconds, board_size=8, threads=None):
    """Scalar restatement of the reference rules engine (oracle/, the per-cell
    8-direction ray walk of othello.py:273-343) with the same random policy and
    auto-reset, one independent batch of boards per host thread (the ctypes
    call releases the GIL); a bounded sample of about `seconds` CPU-seconds
    (at least 2 s of wall time)."""
    import concurrent.futures
    import threading

    from oracle import oracle
    T = threads or cpu_threads()
    E, chunk = 1024, 16
    wall = max(2.0, seconds / T)
    flags = oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET
    start = threading.Barrier(T + 1)

    def worker(k):
        s = oracle.reset(board_size, E)
        plies = 0
        start.wait()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < wall:
            oracle.rollout(s, flags, 0, chunk, seed=0, id_base=k * E, ply0=plies, record=False)
            plies += chunk
        return plies, time.perf_counter() - t0

    with concurrent.futures.ThreadPoolExecutor(T) as ex:
        futs = [ex.submit(worker, k) for k in range(T)]
        start.wait()
        res = [f.result() for f in futs]
    steps = sum(E * p for p, _ in res)
    dt = max(t for _, t in res)
    return {"value": steps / dt, "unit": "env-steps/s", "cores": T, "kind": "port",
            "per_core": steps / dt / T,
            "sample": "%d threads x %d boards of random play, %dx%d, auto-reset, %d env-steps in %.1f s: "
                      "oracle/othello_oracle.c scalar ray-scan restatement of othello.py (same per-cell "
                      "8-direction walk as the reference), one batch per thread"
                      % (T, E, board_size, board_size, steps, dt)}


# VALU issue peak: 256 CUs x 4 SIMD32 x one wave64 instruction per 2 cycles at 2.4 GHz
VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2


def load_pmc(workload):
    """The rocprofv3 PMC summary of this workload committed under profiles/
    (tools/pmc_profile.sh + tools/pmc_summarize.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(workload)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=65536, help="boards per GPU")
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--policy", default="random", choices=["random", "greedy", "maximin1", "maximin2", "maximin3"])
    ap.add_argument("--plies-per-launch", type=int, default=None)
    ap.add_argument("--no-record", action="store_true", help="do not store per-ply action/reward/done")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-ply", action="store_true", help="skip the one-ply-per-launch side measurement")
    ap.add_argument("--no-masked", action="store_true", help="skip the masked-categorical side measurement")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test hooks for rehearsing the multi-process path on a one-GPU box:
    # OTH_BENCH_DEVICE pins every rank to one device, OTH_BENCH_BACKEND=gloo
    gpu = int(os.environ.get("OTH_BENCH_DEVICE", local))
    backend = os.environ.get("OTH_BENCH_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd.distributed import gather_wdl, shard
    from gymothelloenv_amd.vec_env import nwords

    E, n = args.envs, args.board_size
    W = nwords(n)
    P = args.plies_per_launch or (100 if args.policy == "random" else 10)
    steps = max(P, (args.steps // P) * P)
    warm = max(P, (args.warmup // P) * P) if args.warmup > 0 else 0
    launches = steps // P
    record = not args.no_record
    base, _ = shard(E * world, world, rank)  # weak scaling: E boards per GPU, global ids rank*E ...
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, env_id_base=base,
                        initial_rand_steps=10 if args.policy == "greedy" else 0, device=dev)
    env.reset()
    acts = torch.empty(P, E, dtype=torch.int32, device=dev) if record else None
    rews = torch.empty(P, E, dtype=torch.int32, device=dev) if record else None
    dns = torch.empty(P, E, dtype=torch.uint8, device=dev) if record else None

    def run(k_launches):
        for _ in range(k_launches):
            env.step_policy(args.policy, n_plies=P, actions=acts, rewards=rews, dones=dns, record=record)

    run(warm // P)
    env.counts(reset=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    run(launches)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1)  # HIP events on the launch stream
    wdl = env.counts()
    t = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wdl_total = gather_wdl(wdl).sum(0)  # RCCL all-gather over xGMI: the W/D/L tally
    else:
        wdl_total = wdl
    wall_max = float(t.item())
    wdl_total = [int(x) for x in wdl_total.cpu().tolist()]

    # the same play one ply per launch: every ply's state round-trips HBM (the
    # north-star kernel shape); reported beside the headline, not as `value`
    single = None
    if not args.no_single_ply and world == 1:
        a1 = torch.empty(1, E, dtype=torch.int32, device=dev)
        r1 = torch.empty(1, E, dtype=torch.int32, device=dev)
        d1 = torch.empty(1, E, dtype=torch.uint8, device=dev)
        for _ in range(50):
            env.step_policy(args.policy, n_plies=1, actions=a1, rewards=r1, dones=d1)
        torch.cuda.synchronize()
        k1 = 500
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k1):
            env.step_policy(args.policy, n_plies=1, actions=a1, rewards=r1, dones=d1)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / k1
        b1 = algorithmic_bytes_per_launch(E, W, 1, True)
        single = {"value": E / (us * 1e-6), "unit": "env-steps/s", "avg_launch_us": us,
                  "algorithmic_bytes_per_launch": b1, "achieved_GBps": b1 / (us * 1e-6) / 1e9,
                  "steps": k1}

    # side measurement: the learners' masked categorical (csrc/masked.hip) over
    # 4,194,304 boards' fp32 logits (1.1 GB: beyond the 256 MiB Infinity Cache)
    masked = None
    if not args.no_masked and world == 1:
        from gymothelloenv_amd import masked_sample
        Em, nn = 4194304, n * n
        g = torch.Generator(device=dev).manual_seed(0)
        logits = torch.randn(Em, nn, device=dev, generator=g)
        legal = env.legal_mask().repeat((Em + E - 1) // E, 1)[:Em].contiguous()
        outs = [torch.empty(Em, dtype=torch.int32, device=dev)] + \
            [torch.empty(Em, dtype=torch.float32, device=dev) for _ in range(2)]
        lib = env._lib
        import ctypes
        args_m = lambda c: (n, Em, ctypes.c_void_p(logits.data_ptr()), nn, ctypes.c_void_p(legal.data_ptr()),
                            None, 0, 0, c, 0, *[ctypes.c_void_p(o.data_ptr()) for o in outs],
                            ctypes.c_void_p(stream.cuda_stream))
        for c in range(3):
            lib.oth_masked_sample(*args_m(c))
        torch.cuda.synchronize()
        km = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for c in range(km):
            lib.oth_masked_sample(*args_m(c))
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / km
        bm = Em * (4 * nn + 8 * W + 12)
        masked = {"kernel": "k_masked", "boards": Em, "avg_launch_us": us, "algorithmic_bytes_per_launch": bm,
                  "achieved_GBps": bm / (us * 1e-6) / 1e9, "frac_hbm_peak": bm / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS,
                  "boards_per_s": Em / (us * 1e-6)}
        del logits, legal, outs

    if rank == 0:
        total_steps = E * world * steps
        value = total_steps / wall_max
        avg_launch_s = kern_ms / 1e3 / launches
        bytes_launch = algorithmic_bytes_per_launch(E, W, P, record)
        achieved = bytes_launch / avg_launch_s / 1e9
        workload = "%s-play-%dx%d-E%d-P%d" % (args.policy, n, n, E, P)
        if not record:
            workload += "-norecord"
        pmc = load_pmc(workload)
        out = {
            "metric": METRIC if args.policy == "random" else "env-steps/sec (%s policy on device)" % args.policy,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warm,
            "ms_per_step": wall_max / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (standard opening, Philox random play, auto-reset)",
            "config": {"workload": workload, "boards_per_gpu": E, "board_size": n,
                       "global_boards": E * world, "plies_per_launch": P, "policy": args.policy,
                       "per_ply_outputs_stored": record, "parallelism": "dp%d (independent shards)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "kernel": "k_play<%d,%s>" % (n, args.policy), "avg_launch_us": avg_launch_s * 1e6,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "valu": None if not pmc or not pmc.get("valu_insts_per_launch") else {
                             "achieved_wave_insts_per_s": pmc["valu_insts_per_launch"] / avg_launch_s,
                             "peak_wave_insts_per_s": VALU_PEAK_WAVE_INSTS,
                             "frac": pmc["valu_insts_per_launch"] / avg_launch_s / VALU_PEAK_WAVE_INSTS,
                             "note": "the kernel's real limiter: integer VALU issue (one wave per SIMD at "
                                     "65,536 boards), see DESIGN.md"}},
            "wdl": {"black_wins": wdl_total[0], "draws": wdl_total[1], "white_wins": wdl_total[2]},
            "single_ply_launches": single,
            "masked_sample": masked,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, n)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
