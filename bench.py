#!/usr/bin/env python3
"""Benchmark: env-steps/s of on-device random play on 8x8 boards (BASELINE.json
`metric`; config 2 at one GPU, config 4's shards at N GPUs).

Units:
  * env-step = one ply applied to one board (one OthelloBaseEnv.step,
    othello.py:412-462, pass resolution included); the mover
    picks uniformly among its possible_moves (RandomPolicy,
    simple_policies.py:37-41) from a Philox stream; finished games auto-reset.
  * bench step = one rollout segment: `--plies-per-step` P (default 100) plies
    over every board of the shard, one k_play launch (boards kept in registers
    between plies; every ply's action / reward / done stored to HBM).
`--steps K --warmup W` run exactly W untimed and K timed bench steps.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE set, before
the parent touches the GPU) and exits with their status.  Boards per GPU:
65,536 at one GPU (config 2), 131,072 at N > 1 (config 4: 1,048,576 over 8);
`--envs` / `--global-envs` override.  Boards are sharded by global env id
(ShardedVecOthelloEnv); the only exchange is the W/D/L all-gather (RCCL).

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel
(k_play<8, random>) at SURVEY.md §8(d)'s algorithmic bytes per env-step
(40W + 11 = 51 B at 8x8) x env-steps per launch over its average launch time
(HIP events on the launch stream); `traffic` is the measured HBM bytes per
launch from the rocprofv3 PMC summary committed under profiles/; the kernel's
binding limit is integer VALU issue (`valu`).  `cpu_baseline` times the
bitboard CPU engine (oracle/cpu_bitboard.cpp: the kernels' rules templates
compiled for the host) and the scalar restatement of othello.py's ray walk
(oracle/othello_oracle.c) on the host cores over bounded samples.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMDs x one wave64 instruction per 2 cycles at 2.4 GHz
VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2
# ...and the ceiling with ONE wave per SIMD (65,536 boards = 1,024 waves on 1,024 SIMDs): a
# lone wave issues at most one VALU instruction per 4 cycles (tools/ubench_valu3.hip,
# profiles/r06/h; the play kernels' SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU = 4.0)
VALU_LONE_WAVE_CYCLES = 4.0
METRIC = "env-steps/sec (random policy, 65,536×8×8 boards) at 1/2/4/8 GPUs; HBM GB/s vs peak"
CONFIG2_BOARDS = 65536
CONFIG4_BOARDS_PER_GPU = 131072


def step_bytes(W):
    """algorithmic HBM bytes per env-step, 40W + 11 (51 at W = 1):
    state 16W + flags 1 + action 4 in; state 16W + flags 1 + legal 8W + reward 4 + done 1 out."""
    return 40 * W + 11


def fused_bytes_per_launch(E, W, plies, record=True):
    """HBM bytes one fused k_play launch moves: the board state in and out once
    (boards 16W + legal 8W + meta 2, each way) plus per ply action (4), reward (4)
    and done (1) of every board.  Compare with the PMC `traffic`."""
    return E * (2 * (16 * W + 8 * W + 2) + plies * ((4 + 4 + 1) if record else 0))


def cpu_threads():
    """(threads to use, affinity cores, what capped it): every core of the
    affinity set unless the job's thread budget is smaller --
    on the GPU box OMP_NUM_THREADS is the lease's CPU share, while the affinity
    set shows the whole host's cores."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and 0 < int(cap) < n:
        return int(cap), n, "OMP_NUM_THREADS=%s (the job's CPU share)" % cap
    return n, n, None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _timed_threads(T, wall, work):
    """Run work(k, deadline_fn) on T threads started together; returns
    (sum of env-steps, max seconds)."""
    import concurrent.futures
    import threading
    start = threading.Barrier(T + 1)

    def worker(k):
        start.wait()
        t0 = time.perf_counter()
        steps = work(k, lambda: time.perf_counter() - t0 < wall)
        return steps, time.perf_counter() - t0

    with concurrent.futures.ThreadPoolExecutor(T) as ex:
        futs = [ex.submit(worker, k) for k in range(T)]
        start.wait()
        res = [f.result() for f in futs]
    return sum(s for s, _ in res), max(t for _, t in res)


def cpu_baseline(seconds, board_size=8, threads=None):
    """Two CPU engines on the host cores, one independent batch of boards per
    thread (ctypes calls release the GIL), each a bounded sample of about
    `seconds` CPU-seconds (at least 2 s of wall time):
      * bitboard (the headline CPU figure, "best CPU" of SURVEY.md §8(d)):
        oracle/cpu_bitboard.cpp, the kernels' shift/mask rules compiled with g++;
      * scalar port: oracle/othello_oracle.c, the per-cell 8-direction ray walk
        of othello.py:273-343 (the reference's algorithm).
    Both play random moves from the device's Philox stream with auto-reset."""
    from oracle import oracle
    oracle.lib(), oracle.bb_lib()  # loaded (and rebuilt if stale) before any timing
    T, affinity, capped_by = cpu_threads()
    T = threads or T
    wall = max(2.0, seconds / T)
    flags = oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET
    E, chunk = 1024, 16

    def bb_work(k, more):
        s, steps, ply = oracle.reset(board_size, E), 0, 0
        while more():
            steps += oracle.bb_rollout(s, chunk, id_base=k * E, ply0=ply, record=False)[4]
            ply += chunk
        return steps

    def scalar_work(k, more):
        s, ply = oracle.reset(board_size, E), 0
        while more():
            oracle.rollout(s, flags, 0, chunk, seed=0, id_base=k * E, ply0=ply, record=False)
            ply += chunk
        return E * ply

    bb_steps, bb_dt = _timed_threads(T, wall, bb_work)
    sc_steps, sc_dt = _timed_threads(T, wall, scalar_work)
    model = cpu_model()
    return {"value": bb_steps / bb_dt, "unit": "env-steps/s", "cores": T, "kind": "port",
            "affinity_cores": affinity, "cores_capped_by": capped_by,
            "per_core": bb_steps / bb_dt / T, "cpu_model": model,
            "sample": "%d threads x %d boards of random play, %dx%d, auto-reset, %d env-steps in %.1f s on %s: "
                      "oracle/cpu_bitboard.cpp (bitboard.hpp's shift/mask rules compiled for the host, g++ -O3), "
                      "one batch per thread" % (T, E, board_size, board_size, bb_steps, bb_dt, model),
            "scalar_port": {"value": sc_steps / sc_dt, "unit": "env-steps/s", "cores": T, "kind": "port",
                            "per_core": sc_steps / sc_dt / T,
                            "sample": "%d threads x %d boards, %d env-steps in %.1f s: oracle/othello_oracle.c "
                                      "scalar ray-scan restatement of othello.py:273-343" % (T, E, sc_steps, sc_dt)}}


def load_pmc(workload):
    """The rocprofv3 PMC summary of this workload committed under profiles/
    (tools/pmc_profile.sh / tools/gpu_prof_configs.sh + tools/pmc_summarize.py),
    or None."""
    for f in ("pmc_traffic.json", "pmc_configs.json"):
        try:
            rec = json.load(open(os.path.join(ROOT, "profiles", f))).get(workload)
        except Exception:
            rec = None
        if rec:
            return rec
    return None


def pmc_ref(workload, plies=1):
    """A compact reference to the committed PMC record of `workload` (its
    profiles/ path, the HBM bytes and VALU wave-instructions per launch, VALU
    per wave and ply), or None: the bench line names the record, it does not
    inline it."""
    rec = load_pmc(workload)
    if not rec:
        return None
    out = {"source": rec.get("source"), "hbm_bytes_per_launch": _r(rec.get("hbm_bytes_per_launch"))}
    if rec.get("valu_insts_per_launch") and rec.get("waves_per_launch"):
        out["valu_per_wave_ply"] = _r(rec["valu_insts_per_launch"] / rec["waves_per_launch"] / plies)
    return out


def _r(x, digits=4):
    """x to `digits` significant digits (keeps the one JSON line short)."""
    if x is None or isinstance(x, (bool, str)):
        return x
    if isinstance(x, int):
        return x
    return float("%.*g" % (digits, x))


def play_kernel_name(n, policy, record):
    """The kernel oth_step_policy launches for this configuration (kernels_n.hip
    launch_k_play): the restructured auto-reset kernels when every per-ply
    output is stored, else the generic k_play."""
    if record and policy in ("random", "greedy") and n <= 8:
        return "k_play_rand<%d,%s>" % (n, policy)
    if record and policy == "random":
        return "k_play_rand_w<%d>" % n
    return "k_play<%d,%s>" % (n, policy)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50, help="timed bench steps (rollout segments)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed bench steps")
    ap.add_argument("--plies-per-step", type=int, default=None,
                    help="plies per bench step = per k_play launch (default 100 random, 10 otherwise)")
    ap.add_argument("--envs", type=int, default=None, help="boards per GPU")
    ap.add_argument("--global-envs", type=int, default=None, help="boards over all GPUs")
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--policy", default="random", choices=["random", "greedy", "maximin1", "maximin2", "maximin3"])
    ap.add_argument("--no-record", action="store_true", help="do not store per-ply action/reward/done")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side", action="store_true", help="skip the side measurements")
    ap.add_argument("--dry-run", action="store_true",
                    help="ranks, process group and shard plan only (no GPU call); for CPU tests")
    return ap.parse_args(argv)


def plan(args, world, rank):
    """Boards of this rank: (global_envs, env_id_base, n_local, plies per step)."""
    if args.global_envs is not None and args.envs is not None:
        raise SystemExit("give --envs or --global-envs, not both")
    if args.global_envs is not None:
        G = args.global_envs
    else:
        per = args.envs if args.envs is not None else (CONFIG2_BOARDS if world == 1 else CONFIG4_BOARDS_PER_GPU)
        G = per * world
    from gymothelloenv_amd.distributed import shard
    base, n_local = shard(G, world, rank)
    if n_local <= 0:
        raise SystemExit("rank %d has no boards (global %d over %d ranks)" % (rank, G, world))
    P = args.plies_per_step or (100 if args.policy == "random" else 10)
    if args.steps <= 0 or args.warmup < 0 or P <= 0:
        raise SystemExit("need --steps > 0, --warmup >= 0, --plies-per-step > 0")
    return G, base, n_local, P


def spawn(argv, n):
    """Start n ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    set) without touching the GPU here; return the first non-zero exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    # poll every rank: one that dies makes the survivors wait in a collective
    # until its timeout, so end them at once and report the failure
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn(argv, args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    G, base, E, P = plan(args, world, rank)

    import torch
    import torch.distributed as dist
    # test hooks: OTH_BENCH_BACKEND=gloo (CPU tests, or rehearsing N ranks on one
    # GPU), OTH_BENCH_DEVICE pins every rank to one device
    backend = os.environ.get("OTH_BENCH_BACKEND", "nccl")
    gpu = int(os.environ.get("OTH_BENCH_DEVICE", local))
    shared = "OTH_BENCH_DEVICE" in os.environ and world > 1  # every rank on one device (a rehearsal)
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            mine = torch.tensor([rank, base, E], dtype=torch.int64)
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            rows = [p.tolist() for p in parts]
            dist.destroy_process_group()
        else:
            rows = [[rank, base, E]]
        if rank == 0:
            rec = make_record(args, world, G, E, P, args.board_size, not args.no_record, None, None, None,
                              shared_device=shared, pmc={})
            rec.update({"dry_run": True, "world": world, "global_envs": G, "plies_per_step": P, "shards": rows})
            print(json.dumps(rec), flush=True)
        return 0
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from gymothelloenv_amd.distributed import ShardedVecOthelloEnv, gather_wdl
    from gymothelloenv_amd.vec_env import nwords

    n = args.board_size
    W = nwords(n)
    record = not args.no_record
    env = ShardedVecOthelloEnv(G, rank=rank, world=world, board_size=n, auto_reset=True, seed=0,
                               initial_rand_steps=10 if args.policy == "greedy" else 0, device=dev)
    assert env.num_envs == E and env.env_id_base == base
    env.reset()
    acts = torch.empty(P, E, dtype=torch.int32, device=dev) if record else None
    rews = torch.empty(P, E, dtype=torch.int32, device=dev) if record else None
    dns = torch.empty(P, E, dtype=torch.uint8, device=dev) if record else None

    def run(k):
        for _ in range(k):
            env.step_policy(args.policy, n_plies=P, actions=acts, rewards=rews, dones=dns, record=record)

    run(args.warmup)
    env.counts(reset=True)
    stream = torch.cuda.current_stream(dev)
    solo = None
    if world > 1:
        # rank 0's shard timed alone on a twin handle while the other ranks wait
        # (the same-shard one-GPU reference of the scaling curve; the twin keeps
        # the measured handles' games, and so the W/D/L, independent of it)
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 0:
            twin = ShardedVecOthelloEnv(G, rank=rank, world=world, board_size=n, auto_reset=True, seed=0,
                                        initial_rand_steps=10 if args.policy == "greedy" else 0, device=dev)
            twin.reset()
            for _ in range(args.warmup):
                twin.step_policy(args.policy, n_plies=P, actions=acts, rewards=rews, dones=dns, record=record)
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            for _ in range(args.steps):
                twin.step_policy(args.policy, n_plies=P, actions=acts, rewards=rews, dones=dns, record=record)
            torch.cuda.synchronize()
            dt = time.perf_counter() - s0
            solo = {"value": E * P * args.steps / dt, "unit": "env-steps/s", "boards": E,
                    "ms_per_step": dt / args.steps * 1e3, "note": "rank 0's shard alone, other ranks idle"}
            twin.close()
        dist.barrier()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    run(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1)  # HIP events on the launch stream
    wdl = env.counts()
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall_max = float(t.item())
        wdl_total = gather_wdl(wdl).sum(0)  # RCCL all-gather over xGMI: the W/D/L tally
    else:
        wall_max, wdl_total = wall, wdl
    wdl_total = [int(x) for x in wdl_total.cpu().tolist()]

    side = {}
    if not args.no_side and world == 1 and rank == 0:
        side = side_measurements(env.env, args.policy, E, n, W, dev, stream, P=P, bufs=(acts, rews, dns),
                                 burst_us=kern_ms * 1e3 / args.steps)

    if rank == 0:
        out = make_record(args, world, G, E, P, n, record, wall_max, kern_ms, wdl_total, solo=solo,
                          shared_device=shared)
        out.update(side)
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, n)
        if side:
            out["side_summary"] = side_summary(side, out)  # last: a truncated tail still shows it
        print(json.dumps(out, separators=(",", ":")), flush=True)  # compact: the driver keeps a 2,000-char tail
    env.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def make_record(args, world, G, E, P, n, record, wall_max, kern_ms, wdl_total, solo=None, shared_device=False,
                pmc=None):
    """The JSON line rank 0 prints.  wall_max: max over ranks of the timed
    region's wall time (s); kern_ms: rank 0's HIP-event time of the K launches
    (None in --dry-run, which prints the same keys with null numbers)."""
    from gymothelloenv_amd.vec_env import nwords
    W = nwords(n)
    env_steps = G * P * args.steps
    bps = step_bytes(W)
    alg_launch = E * P * bps
    avg_launch_s = kern_ms / 1e3 / args.steps if kern_ms else None
    achieved = alg_launch / avg_launch_s / 1e9 if avg_launch_s else None
    workload = "%s-play-%dx%d-E%d-P%d" % (args.policy, n, n, E, P)
    if not record:
        workload += "-norecord"
    pmc = pmc if pmc is not None else load_pmc(workload)
    valu = None
    if pmc and pmc.get("valu_insts_per_launch") and avg_launch_s:
        rate = pmc["valu_insts_per_launch"] / avg_launch_s
        waves = -(-E // 64)
        lone = None
        if waves <= 1024:  # at most one wave per SIMD: the lone wave's issue interval bounds it
            lone = waves * 2.4e9 / VALU_LONE_WAVE_CYCLES
        valu = {"achieved_wave_insts_per_s": rate, "peak_wave_insts_per_s": VALU_PEAK_WAVE_INSTS,
                "frac": rate / VALU_PEAK_WAVE_INSTS,
                "lone_wave_peak_wave_insts_per_s": lone,
                "lone_wave_frac": rate / lone if lone else None,
                # SQ_INSTS_VALU counts wave-instructions, each serving 64 boards: x 64 / board-plies
                # is the length of one board's (one lane's) VALU instruction stream per ply
                "valu_insts_per_board_ply": pmc["valu_insts_per_launch"] * 64 / (E * P),
                "wave_insts_per_launch": pmc["valu_insts_per_launch"],
                "source": "SQ_INSTS_VALU per launch from %s, this run's launch time" % pmc.get("source", "?")}
    metric = METRIC if args.policy == "random" else "env-steps/sec (%s policy on device, %dx%d)" % (args.policy, n, n)
    config_name = "config2" if (world == 1 and G == CONFIG2_BOARDS) else \
        ("config4" if (world == 8 and G == 8 * CONFIG4_BOARDS_PER_GPU) else "custom")
    value = env_steps / wall_max if wall_max else None
    out = {
        "metric": metric,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": 1 if shared_device else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max / args.steps * 1e3 if wall_max else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (standard opening, Philox random play, auto-reset)",
        "config": {"workload": workload, "baseline_config": config_name, "boards_per_gpu": E,
                   "global_boards": G, "board_size": n, "plies_per_step": P,
                   "env_steps_per_step": G * P, "policy": args.policy, "per_ply_outputs_stored": record,
                   "parallelism": "dp%d (independent shards, W/D/L all-gather only)" % world},
        "roofline": {"bound": "valu-issue", "limiter": "integer VALU issue at one wave per SIMD (see valu); "
                                                         "achieved / frac are against HBM",
                     "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS if achieved else None,
                     "achieved_kind": "equivalent bandwidth: SURVEY §8(d)'s algorithmic bytes over the launch time; "
                                      "the fused launch keeps boards in registers, so HBM moves `traffic` only",
                     "moved_GBps": pmc["hbm_bytes_per_launch"] / avg_launch_s / 1e9 if pmc and avg_launch_s else None,
                     "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                     "traffic_source": pmc.get("source") if pmc else None,
                     "kernel": play_kernel_name(n, args.policy, record),
                     "avg_launch_us": avg_launch_s * 1e6 if avg_launch_s else None,
                     "launches_timed": args.steps,
                     "algorithmic_bytes_per_env_step": bps,
                     "algorithmic_bytes_per_launch": alg_launch,
                     "fused_bytes_per_launch": fused_bytes_per_launch(E, W, P, record),
                     "valu": valu,
                     "note": "achieved/frac: SURVEY §8(d) bytes (40W+11 per env-step) over the launch time; "
                             "traffic: PMC FETCH_SIZE x2 + WRITE_SIZE per launch of the final build (the fused "
                             "kernel keeps boards in registers between plies); the limiter is integer VALU issue"},
        "wdl": {"black_wins": wdl_total[0], "draws": wdl_total[1], "white_wins": wdl_total[2]}
        if wdl_total is not None else None,
    }
    if world > 1 or shared_device:
        # SCALE reading aid: N > 1 runs config 4's 131,072 boards per GPU (two waves per SIMD),
        # N = 1 config 2's 65,536 (one wave per SIMD), so compare per_gpu_value with
        # single_gpu_same_shard (rank 0's shard timed alone, the other ranks idle at a barrier)
        out["per_gpu_value"] = value / world if value else None
        out["single_gpu_same_shard"] = solo
        out["ranks"] = world
        out["shared_device"] = bool(shared_device)
    return out


def _time_launches(stream, fn, k):
    """Average time of k back-to-back launches fn(i) on `stream` (HIP events)."""
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for i in range(k):
        fn(i)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


def step_external(E, n, dev, stream, plies=64):
    """oth_step (OthelloBaseEnv.step, othello.py:412-462) with external device
    actions, one launch per ply (the north star's step(action) path: the state
    round-trips HBM every ply).  The actions are P plies of recorded on-device
    random play (all legal, auto-reset), replayed from the recording's start
    state; the replay must end in the recording's state (checked)."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd.vec_env import nwords
    W = nwords(n)
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev)
    env.step_policy("random", n_plies=30, record=False)  # a mid-game mix of boards
    b0, m0, l0 = env.get_state()
    ply0 = env.ply_counter
    acts = torch.empty(plies, E, dtype=torch.int32, device=dev)
    rec_r = torch.empty(plies, E, dtype=torch.int32, device=dev)
    rec_d = torch.empty(plies, E, dtype=torch.uint8, device=dev)
    env.step_policy("random", n_plies=plies, actions=acts, rewards=rec_r, dones=rec_d)
    b1, m1, l1 = env.get_state()
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)

    rows = list(acts.unbind(0))  # one action tensor per ply, as a policy hands them over (no indexing in the loop)

    def replay(i):
        env.step(rows[i], rewards=rew, dones=don, observe=False)

    def matches():
        b2, m2, l2 = env.get_state()
        return bool(torch.equal(b1, b2) and torch.equal(m1, m2) and torch.equal(l1, l2) and
                    torch.equal(rew, rec_r[-1]) and torch.equal(don, rec_d[-1]))
    eager_us = None
    for _ in range(2):  # eager launches (host launch path included); the first warms up
        env.set_state(b0, m0, l0)
        env.ply_counter = ply0
        eager_us = _time_launches(stream, replay, plies)
    same = matches()
    # the same P launches replayed from a HIP graph: the kernels back to back, no host in the loop
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), env.graph_region():
        for i in range(plies):
            replay(i)
    reps = []
    for _ in range(5):  # the median of five replays (the first on a fresh box runs at lower clocks)
        env.set_state(b0, m0, l0)
        reps.append(_time_launches(stream, lambda i: g.replay(), 1) / plies)
    us = statistics.median(reps)
    same = same and matches()
    env.close()
    bps = step_bytes(W)
    gbs = E * bps / (us * 1e-6) / 1e9
    return {"kernel": "k_ply_step<%d>" % n if W == 1 else "k_step<%d>" % n, "boards": E, "value": E / (us * 1e-6),
            "unit": "env-steps/s", "avg_launch_us": us, "launches": plies,
            "timing": "HIP graph of the %d launches, HIP events around the replay, median of 5" % plies,
            "eager_avg_launch_us": eager_us,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBPS, "algorithmic_bytes_per_env_step": bps},
            "replay_equals_recording": same}


def _graph_us(env, start, fn, k, stream):
    """Median of 5 replays of a HIP graph of fn(0 .. k-1) (inside a graph
    region: fresh Philox counters every replay), each replay from the state
    `start`; us per call."""
    import torch
    g = torch.cuda.CUDAGraph()
    env.set_state(*start)
    with torch.cuda.graph(g), env.graph_region():
        for i in range(k):
            fn(i)
    reps = []
    for _ in range(5):
        env.set_state(*start)
        reps.append(_time_launches(stream, lambda i: g.replay(), 1) / k)
    del g
    return statistics.median(reps)


def step_observe_lines(E, n, dev, stream, plies=32):
    """The step with its observation from one launch, against the two-launch
    form and the parts alone, graphed (plies calls, median of 5 replays, each
    from the same mid-game state):
      * oth_step_observe: OthelloBaseEnv.step's (obs, reward, done) tuple
        (othello.py:412-462) with the int64 get_observation (:363-378), replaying
        recorded random moves;
      * oth_sample_step_observe: the learners' ply -- Policy.act's masked sample
        (model.py:60-99) + step + util.make_state f32 (util.py:48-74), the next
        input of the policy network.
    frac: SURVEY §8(d)'s 51 B per env-step plus the observation written (512 B
    int64 board / 1,024 B f32 make_state per 8x8 board), plus the logits read
    and the sample written (4N² + 12 B) for the learners' ply, over the time."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd.vec_env import nwords
    W, NN = nwords(n), n * n
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev)
    env.step_policy("random", n_plies=30, record=False)
    start = env.get_state()
    acts = env.step_policy("random", n_plies=plies)[0]
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    ob = torch.empty(E, n, n, dtype=torch.int64, device=dev)
    ms = torch.empty(E, 4, n, n, dtype=torch.float32, device=dev)
    ms8 = torch.empty(E, 4, n, n, dtype=torch.int8, device=dev)
    ms16 = torch.empty(E, 4, n, n, dtype=torch.bfloat16, device=dev)
    a = torch.empty(E, dtype=torch.int32, device=dev)
    lp = torch.empty(E, dtype=torch.float32, device=dev)
    en = torch.empty(E, dtype=torch.float32, device=dev)
    logits = torch.randn(E, NN, device=dev, generator=torch.Generator(device=dev).manual_seed(0))

    def ss(i, obs=None):
        return env.sample_step(logits, actions=a, log_probs=lp, entropy=en, rewards=rew, dones=don,
                               **({"observe": "make_state", "obs": obs} if obs is not None else {}))
    t = {"step_board_fused": lambda i: env.step(acts[i], rewards=rew, dones=don, obs=ob),
         "step_board_split": lambda i: (env.step(acts[i], rewards=rew, dones=don, observe=False),
                                        env.observe("board", torch.int64, out=ob)),
         "step_only": lambda i: env.step(acts[i], rewards=rew, dones=don, observe=False),
         "sample_step_make_state_fused": lambda i: ss(i, ms),
         "sample_step_make_state_split": lambda i: (ss(i), env.observe("make_state", torch.float32, out=ms)),
         "sample_step_only": lambda i: ss(i),
         # make_state in int8 / bfloat16 (exact for its 0 / 1 planes): a quarter / half the bytes
         "sample_step_make_state_i8_fused": lambda i: ss(i, ms8),
         "sample_step_make_state_bf16_fused": lambda i: ss(i, ms16),
         # what an f32 / bf16 consumer pays to widen the int8 planes into its first layer's input
         "cast_i8_to_f32": lambda i: ms.copy_(ms8),
         "cast_i8_to_bf16": lambda i: ms16.copy_(ms8)}
    us = {k: _graph_us(env, start, fn, plies, stream) for k, fn in t.items()}
    env.close()
    step_b = 40 * W + 11
    b_board = E * (step_b + 8 * NN)

    def b_ply(esize):  # the learners' ply: logits in, the sample out, the step, make_state written
        return E * (4 * NN + 12 + step_b + 4 * esize * NN)
    b_ms = b_ply(4)

    def frac(b, u):
        return _r(b / (u * 1e-6) / 1e9 / HBM_PEAK_GBPS)
    return {"boards": E, "board_size": n,
            "us": {k: _r(v) for k, v in us.items()},
            "step_board": {"kernel": "k_ply_step_obs<%d>" % n if W == 1 else "k_step<%d> + k_observe_w" % n,
                           "us_per_ply": _r(us["step_board_fused"]),
                           "two_launch_us": _r(us["step_board_split"]),
                           "algorithmic_bytes_per_board": step_b + 8 * NN,
                           "frac": frac(b_board, us["step_board_fused"]),
                           "pmc": pmc_ref("step-observe-board-int64-%dx%d-E%d" % (n, n, E))},
            "sample_step_make_state": {"kernel": "k_sample_step2<%d> + obs tail" % n,
                                       "us_per_ply": _r(us["sample_step_make_state_fused"]),
                                       "two_launch_us": _r(us["sample_step_make_state_split"]),
                                       "algorithmic_bytes_per_board": 4 * NN + 12 + step_b + 16 * NN,
                                       "frac": frac(b_ms, us["sample_step_make_state_fused"]),
                                       "pmc": pmc_ref("sample-step-make-state-f32-%dx%d-E%d" % (n, n, E))},
            "sample_step_make_state_narrow": {
                "kernel": "k_sample_step2<%d> + obs tail" % n,
                "i8_us_per_ply": _r(us["sample_step_make_state_i8_fused"]),
                "i8_bytes_per_board": 4 * NN + 12 + step_b + 4 * NN,
                "i8_frac": frac(b_ply(1), us["sample_step_make_state_i8_fused"]),
                "bf16_us_per_ply": _r(us["sample_step_make_state_bf16_fused"]),
                "bf16_bytes_per_board": 4 * NN + 12 + step_b + 8 * NN,
                "bf16_frac": frac(b_ply(2), us["sample_step_make_state_bf16_fused"]),
                "cast_i8_to_f32_us": _r(us["cast_i8_to_f32"]), "cast_i8_to_bf16_us": _r(us["cast_i8_to_bf16"]),
                "note": "make_state is 0 / 1: exact in int8 and bfloat16; the cast lines are torch's copy_ of the "
                        "int8 planes into an f32 / bf16 tensor of the same shape (a consumer widening them)"},
            "timing": "HIP graph of %d calls from one mid-game state, median of 5 replays" % plies}


def sustained_line(env, policy, P, acts, rews, dns, stream, burst_launch_us, seconds=2.0):
    """The headline launch back to back for about `seconds` (against the timed
    region's short burst, which a clock that drops under sustained load would
    flatter, MI355X_MICROARCH.md 'DVFS give-back').  The effective clock of
    the same sustained run is measured by rocprofv3's GRBM_GUI_ACTIVE in its own
    pass (tools/gpu_sustained_clock.sh) and referenced here."""
    k = max(20, int(seconds / (burst_launch_us * 1e-6)))
    us = _time_launches(stream, lambda i: env.step_policy(policy, n_plies=P, actions=acts, rewards=rews,
                                                          dones=dns), k)
    n = env.board_size
    rec = load_pmc("sustained-%s-play-%dx%d-E%d-P%d" % (policy, n, n, env.num_envs, P))
    return {"launches": k, "seconds": _r(k * us * 1e-6), "avg_launch_us": _r(us),
            "value": _r(env.num_envs * P / (us * 1e-6)), "unit": "env-steps/s",
            "vs_burst": _r(burst_launch_us / us),
            "effective_clock_ghz": _r(rec.get("effective_clock_ghz")) if rec else None,
            "clock_source": rec.get("source") if rec else None}


def side_summary(side, out):
    """The side lines' headline numbers in one compact object, printed LAST on
    the line (a truncated tail still holds them): us per ply (or call), frac of
    HBM, VALU per wave-ply from the committed PMC records."""
    summ = {}

    def pm(x):
        p = ((x.get("roofline") or {}).get("pmc") or {})
        return p.get("valu_per_wave_ply")
    c = side.get("configs", {})
    for x in c.get("config3_greedy", []):
        summ["config3_greedy_P%d" % x["plies_per_launch"]] = {
            "us_per_ply": _r(x["us_per_ply"]), "frac": _r(x["roofline"]["frac"]), "valu_per_wave_ply": pm(x)}
    for x in c.get("config5_random", []):
        summ["config5_random_%dx%d" % (x["board_size"], x["board_size"])] = {
            "us_per_ply": _r(x["us_per_ply"]), "frac": _r(x["roofline"]["frac"]), "valu_per_wave_ply": pm(x)}
    if c.get("config1_single_board"):
        summ["config1_single_board"] = {"us_per_step": _r(c["config1_single_board"]["us_per_step"])}
    for x in side.get("step_external", []):
        summ["step_external_E%d" % x["boards"]] = {"us_per_ply": _r(x["avg_launch_us"]),
                                                   "eager_us": _r(x["eager_avg_launch_us"]),
                                                   "frac": _r(x["roofline"]["frac"])}
    so = side.get("step_observe")
    if so:
        for k in ("step_board", "sample_step_make_state"):
            summ[k] = {"us_per_ply": so[k]["us_per_ply"], "two_launch_us": so[k]["two_launch_us"],
                       "frac": so[k]["frac"]}
        summ["sample_step"] = {"us_per_ply": so["us"]["sample_step_only"]}
        nw = so.get("sample_step_make_state_narrow")
        if nw:
            summ["sample_step_make_state_i8"] = {"us_per_ply": nw["i8_us_per_ply"], "frac": nw["i8_frac"]}
            summ["sample_step_make_state_bf16"] = {"us_per_ply": nw["bf16_us_per_ply"], "frac": nw["bf16_frac"]}
    for x in side.get("othello_env_vs", []):
        summ["othello_env_vs_" + x["opponent"]] = {"us_per_call": _r(x["us_per_call"]),
                                                   "env_steps_per_s": _r(x["env_steps_per_s"])}
    for x in side.get("observe", []):
        summ[x["workload"]] = {"us": _r(x["avg_launch_us"]), "frac": _r(x["roofline"]["frac"])}
    for x in side.get("maximin", []):
        summ["policy_actions_" + x["policy"]] = {"us_per_call": x["us_per_call"], "boards": x["boards"]}
    if side.get("sustained"):
        summ["sustained"] = {k: side["sustained"][k] for k in ("seconds", "avg_launch_us", "vs_burst",
                                                                 "effective_clock_ghz")}
    v = (out.get("roofline") or {}).get("valu") or {}
    summ["headline"] = {"us_per_launch": _r(out["roofline"]["avg_launch_us"]), "frac": _r(out["roofline"]["frac"]),
                        "valu_per_board_ply": _r(v.get("valu_insts_per_board_ply")),
                        "valu_lone_wave_frac": _r(v.get("lone_wave_frac"))}
    return summ


def vs_line(E, n, dev, stream, calls=64, opponent="random", observe=False):
    """OthelloEnv's turn loop on the device (othello.py:151-200; oth_reset_vs /
    oth_step_vs): a greedy protagonist (oth_policy_actions, GreedyPolicy
    simple_policies.py:69-92) against the embedded `opponent` on E boards with
    auto-reset and 0-10-ply random openings (without them every greedy-vs-greedy
    game is the same), the README's evaluation protocol batched.  One call = the
    protagonist's greedy move + its step + the opponent's replies until the
    protagonist is to move again; `calls` calls captured in a HIP graph (median of 5
    replays).  env-steps counted = plies applied (the `plies` output: one
    protagonist ply plus the opponent's)."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=11, device=dev, initial_rand_steps=10)
    env.reset_vs(opponent, protagonist=1)
    plies = []  # each call's plies-applied tensor (graph memory: holds the last replay's values)

    ob = torch.empty(E, n, n, dtype=torch.int64, device=dev) if observe else None

    def call():  # observe: OthelloEnv.step's int64 obs (othello.py:200) from the same launch
        return env.step_vs(env.policy_actions("greedy"), opponent, observe=observe, obs=ob)[3]
    for _ in range(4):
        call()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), env.graph_region():
        for _ in range(calls):
            plies.append(call())
    reps = []
    for _ in range(5):
        reps.append(_time_launches(stream, lambda i: g.replay(), 1) / calls)
    us = statistics.median(reps)
    applied = int(sum(int(p.sum().item()) for p in plies))  # plies of the last replay
    wdl = [int(x) for x in env.counts_vs()]
    env.close()
    return {"workload": "othello-env-vs-%s-%dx%d-E%d%s" % (opponent, n, n, E, "-obs" if observe else ""), "boards": E,
            "opponent": opponent + ("+obs" if observe else ""),
            "kernels": "k_policy_actions<greedy> + k_step_vs%s<%s>" % ("1" if n <= 8 and opponent in ("random", "greedy")
                                                                       else "", opponent),
            "us_per_call": us,
            "plies_per_call": applied / calls, "env_steps_per_s": applied / calls / (us * 1e-6),
            "protagonist_wdl": wdl, "timing": "HIP graph of %d calls, median of 5 replays" % calls}


def maximin_lines(E, n, dev, stream, depths=(2, 3, 4)):
    """MaxiMinPolicy(d).get_action (simple_policies.py:98-163) for every board's
    side to move (oth_policy_actions) on E mid-game boards (25 plies of random
    play): depth 2 one lane per board (maximin_node), depth >= 3 a wave per
    board (k_maximin_wave).  HIP events around `launches` back-to-back launches."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=5, device=dev)
    env.step_policy("random", n_plies=25, record=False)
    out = []
    for d in depths:
        pol = "maximin%d" % d
        env.policy_actions(pol)
        launches = 5 if d >= 4 else 20
        us = _time_launches(stream, lambda i: env.policy_actions(pol), launches)
        out.append({"policy": pol, "boards": E, "board_size": n, "us_per_call": _r(us),
                    "moves_per_s": _r(E / (us * 1e-6)),
                    "kernel": "k_maximin_wave<%d>" % n if d >= 3 else "k_policy_actions<%d,maximin2>" % n})
    env.close()
    return out


def single_ply(env, policy, E, W, dev, stream, k=64):
    """oth_step_policy with one ply per launch (k_ply_rand for random play on
    one-word boards): every board's state through HBM every ply.  k launches
    captured in a HIP graph (a graph region: fresh Philox counters every replay)
    and replayed; eager launches (the host's Python + ctypes path included) beside."""
    import torch
    a1 = torch.empty(1, E, dtype=torch.int32, device=dev)
    r1 = torch.empty(1, E, dtype=torch.int32, device=dev)
    d1 = torch.empty(1, E, dtype=torch.uint8, device=dev)

    def one(i):
        env.step_policy(policy, n_plies=1, actions=a1, rewards=r1, dones=d1)
    for _ in range(20):
        one(0)
    eager_us = _time_launches(stream, one, k)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), env.graph_region():
        for i in range(k):
            one(i)
    us = statistics.median([_time_launches(stream, lambda i: g.replay(), 1) / k for _ in range(5)])
    gbs = E * step_bytes(W) / (us * 1e-6) / 1e9
    return {"boards": E, "value": E / (us * 1e-6), "unit": "env-steps/s", "avg_launch_us": us, "launches": k,
            "timing": "HIP graph of the %d launches, median of 5 replays" % k, "eager_avg_launch_us": eager_us,
            "algorithmic_GBps": gbs, "frac": gbs / HBM_PEAK_GBPS}


def play_line(policy, n, E, P, init_rand, dev, stream, launches=20, warm=3):
    """One oth_step_policy launch of P plies over E boards with auto-reset and
    every per-ply output stored (k_play_rand<N, policy> for N <= 8,
    k_play_rand_w<N> above): BASELINE config 3 (greedy, 8x8, 0..init_rand-ply
    random openings as bench's greedy) and config 5 (random, 6x6 / 10x10).
    HIP events around `launches` back-to-back launches on the launch stream."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd.vec_env import nwords
    W = nwords(n)
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, initial_rand_steps=init_rand, device=dev)
    env.reset()
    acts = torch.empty(P, E, dtype=torch.int32, device=dev)
    rews = torch.empty(P, E, dtype=torch.int32, device=dev)
    dns = torch.empty(P, E, dtype=torch.uint8, device=dev)

    def one(i):
        env.step_policy(policy, n_plies=P, actions=acts, rewards=rews, dones=dns)
    for i in range(warm):
        one(i)
    us = _time_launches(stream, one, launches)
    wdl = [int(x) for x in env.counts().cpu().tolist()]
    env.close()
    bps = step_bytes(W)
    gbs = E * P * bps / (us * 1e-6) / 1e9
    workload = "%s-play-%dx%d-E%d-P%d" % (policy, n, n, E, P)
    return {"workload": workload, "kernel": play_kernel_name(n, policy, True), "boards": E, "board_size": n,
            "plies_per_launch": P, "initial_rand_steps": init_rand, "avg_launch_us": us, "us_per_ply": us / P,
            "value": E * P / (us * 1e-6), "unit": "env-steps/s", "launches_timed": launches, "wdl": wdl,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBPS, "algorithmic_bytes_per_env_step": bps,
                         "fused_bytes_per_launch": fused_bytes_per_launch(E, W, P),
                         "pmc": pmc_ref(workload, P)}}


def observe_bytes(n, E, layout, esize):
    """get_observation / make_state: the (E, planes, N, N) output written once,
    the board words (16W), meta (2) and, for the layouts with a legal plane,
    possible_moves (8W) read once per board."""
    W = (n * n + 63) // 64
    planes = {"board": 1, "board_legal": 2, "make_state": 4, "absolute": 1, "legal": 1}[layout]
    reads = 16 * W + 2 + (8 * W if layout in ("board_legal", "make_state", "legal") else 0)
    return E * (planes * n * n * esize + reads)


def observe_lines(n, sizes, dev, stream, launches=50):
    """oth_observe (k_observe_w) into a preallocated tensor: int64 BOARD (the
    Gym-style get_observation, othello.py:363-378) and f32 MAKE_STATE
    (util.make_state, util.py:48-74), mid-game boards; HIP graph of `launches`
    launches (the short launches back to back), median of 5 replays."""
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    out = []
    for E in sizes:
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=3, device=dev)
        env.step_policy("random", n_plies=25, record=False)
        for layout, dt, esize in (("board", torch.int64, 8), ("make_state", torch.float32, 4)):
            shape = (E, n, n) if layout == "board" else (E, 4, n, n)
            buf = torch.empty(shape, dtype=dt, device=dev)
            for _ in range(3):
                env.observe(layout, dt, out=buf)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(launches):
                    env.observe(layout, dt, out=buf)
            us = statistics.median([_time_launches(stream, lambda i: g.replay(), 1) / launches for _ in range(5)])
            del g
            b = observe_bytes(n, E, layout, esize)
            workload = "observe-%s-%s-%dx%d-E%d" % (layout, str(dt).replace("torch.", ""), n, n, E)
            out.append({"workload": workload, "kernel": "k_observe_w<%d,%s,%s>" % (n, layout, str(dt)),
                        "boards": E, "avg_launch_us": us, "algorithmic_bytes_per_launch": b,
                        "timing": "HIP graph of %d launches, median of 5 replays" % launches,
                        "roofline": {"bound": "hbm", "achieved": b / (us * 1e-6) / 1e9, "peak": HBM_PEAK_GBPS,
                                     "unit": "GB/s", "frac": b / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS,
                                     "pmc": pmc_ref(workload)}})
            del buf
        env.close()
    return out


def config1_line(dev, seconds=0.5):
    """BASELINE config 1: ONE 8x8 board through the drop-in OthelloEnv
    (othello.py:96-214), random protagonist against RandomPolicy, reset after
    each game, for a bounded wall time.  Every step synchronises (the drop-in
    returns host values, as the reference does), so this is the per-call latency
    of the device path, not throughput; the reference's own Python runs
    6.6-8.5 x 10^3 plies/s per core."""
    import contextlib
    import io

    import numpy as np

    from gymothelloenv_amd import OthelloEnv
    from gymothelloenv_amd.policies import RandomPolicy
    rnd = np.random.RandomState(0)
    env = OthelloEnv(white_policy=RandomPolicy(1), black_policy=RandomPolicy(1), protagonist=1, device=dev)
    calls = games = 0
    with contextlib.redirect_stdout(io.StringIO()):  # reset() prints, as the reference's does
        env.reset()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            moves = env.possible_moves
            _, _, done, _ = env.step(moves[rnd.randint(0, len(moves))])
            calls += 1
            if done:
                games += 1
                env.reset()
        dt = time.perf_counter() - t0
    env.close()
    return {"workload": "config1: one 8x8 board, OthelloEnv drop-in, random vs RandomPolicy",
            "env_steps_per_s": calls / dt, "us_per_step": dt / calls * 1e6, "steps": calls, "games": games,
            "note": "each step() synchronises and returns host values (the reference's API); latency, not "
                    "throughput"}


def side_measurements(env, policy, E, n, W, dev, stream, P=None, bufs=None, burst_us=None):
    """Beside the headline (never `value`): the per-step paths with the state
    through HBM every ply -- oth_step with external actions (`step_external`)
    and one-ply launches of the policy (`single_ply_launches`) -- at config 2's
    65,536 boards and config 4's 1,048,576 on one GPU, and the learners' masked
    categorical over 4,194,304 boards' fp32 logits (beyond the 256 MiB MALL)."""
    import ctypes

    import torch

    from gymothelloenv_amd import VecOthelloEnv
    out = {"step_external": [step_external(Eb, n, dev, stream) for Eb in (E, 1048576)]}
    out["step_observe"] = step_observe_lines(E, n, dev, stream)
    # BASELINE configs 3 (greedy, 8x8) and 5 (random, 6x6 and 10x10) at their stated 65,536 boards
    out["configs"] = {"config3_greedy": [play_line("greedy", 8, CONFIG2_BOARDS, P, 10, dev, stream)
                                         for P in (10, 100)],
                      "config5_random": [play_line("random", nb, CONFIG2_BOARDS, 100, 0, dev, stream)
                                         for nb in (6, 10)]}
    out["observe"] = observe_lines(n, (E, 1048576), dev, stream)
    out["configs"]["config1_single_board"] = config1_line(dev)
    out["othello_env_vs"] = [vs_line(E, n, dev, stream, opponent=o) for o in ("random", "greedy", "maximin2")] + \
        [vs_line(E, n, dev, stream, opponent="random", observe=True)]
    out["maximin"] = maximin_lines(E, n, dev, stream)
    big = VecOthelloEnv(1048576, board_size=n, auto_reset=True, seed=0, device=dev)
    big.step_policy(policy, n_plies=20, record=False)
    out["single_ply_launches"] = [single_ply(env, policy, E, W, dev, stream),
                                  single_ply(big, policy, 1048576, W, dev, stream)]
    big.close()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    Em, nn = 4194304, n * n
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(Em, nn, device=dev, generator=g)
    legal = env.legal_mask().repeat((Em + E - 1) // E, 1)[:Em].contiguous()
    outs = [torch.empty(Em, dtype=torch.int32, device=dev)] + \
        [torch.empty(Em, dtype=torch.float32, device=dev) for _ in range(2)]
    lib = env._lib

    def call(c):
        lib.oth_masked_sample(n, Em, ctypes.c_void_p(logits.data_ptr()), nn, ctypes.c_void_p(legal.data_ptr()),
                              None, 0, 0, c, 0, *[ctypes.c_void_p(o.data_ptr()) for o in outs],
                              ctypes.c_void_p(stream.cuda_stream))
    for c in range(3):
        call(c)
    torch.cuda.synchronize()
    km = 20
    e0.record(stream)
    for c in range(km):
        call(c)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / km
    bm = Em * (4 * nn + 8 * W + 12)
    out["masked_sample"] = {"kernel": "k_masked", "boards": Em, "avg_launch_us": us,
                            "algorithmic_bytes_per_launch": bm, "achieved_GBps": bm / (us * 1e-6) / 1e9,
                            "frac_hbm_peak": bm / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS}
    del logits, legal, outs
    if bufs is not None and burst_us:
        out["sustained"] = sustained_line(env, policy, P, *bufs, stream, burst_us)
    return out


if __name__ == "__main__":
    sys.exit(main())
