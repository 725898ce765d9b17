#!/usr/bin/env python3
"""BASELINE configs 3 and 5 and the observation encoders, one workload per
case, for rocprofv3 kernel traces and counter passes (tools/gpu_prof_configs.sh);
prints one JSON line per case with the HIP-event time per launch.

  greedy10 / greedy100   config 3: k_play_rand<8, GREEDY>, 65,536 boards, 10 / 100
                         plies per launch, 0..10-ply random openings (bench.py's greedy)
  rand6 / rand10         config 5: k_play_rand<6, RANDOM> / k_play_rand_w<10>, 65,536 boards,
                         100 plies per launch
  obs                    k_observe_w: int64 BOARD (get_observation) and f32 MAKE_STATE
                         (util.make_state) at 65,536 and 1,048,576 8x8 boards

    python tools/prof_configs.py --cases greedy10,rand6 [--launches 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

PLAY = {"greedy10": ("greedy", 8, 10, 10), "greedy100": ("greedy", 8, 100, 10),
        "rand6": ("random", 6, 100, 0), "rand10": ("random", 10, 100, 0), "rand8": ("random", 8, 100, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="greedy10,greedy100,rand6,rand10,obs")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for case in args.cases.split(","):
        if case in PLAY:
            pol, n, P, init = PLAY[case]
            rec = bench.play_line(pol, n, args.envs, P, init, dev, stream, launches=args.launches)
        elif case == "obs":
            for rec in bench.observe_lines(8, (args.envs, 1048576), dev, stream, launches=args.launches):
                rec["case"] = "obs"
                print(json.dumps(rec), flush=True)
            continue
        else:
            raise SystemExit("unknown case %s" % case)
        rec["case"] = case
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
