#!/usr/bin/env python3
"""The bench's OthelloEnv turn-loop lines (bench.vs_line) alone, for a kernel trace:

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/prof_vs.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    for o in ("random", "greedy"):
        print(json.dumps(bench.vs_line(65536, 8, dev, st, opponent=o)), flush=True)


if __name__ == "__main__":
    main()
