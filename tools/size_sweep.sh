#!/bin/bash
# Board-size sweep of the bench (random play, 65,536 boards, 100 plies per launch)
# plus greedy at 8x8.  Usage on the GPU box: bash tools/size_sweep.sh <outdir>
set -e
OUT=${1:-gpurun_out/sweep}
mkdir -p $OUT
: > $OUT/sweep.jsonl
for n in 4 5 6 7 8 9 10 12 14 16; do
  timeout -k 10 120 python bench.py --board-size $n --steps 1000 --warmup 100 --no-cpu-baseline --no-single-ply --no-masked >> $OUT/sweep.jsonl
done
timeout -k 10 120 python bench.py --policy greedy --steps 1000 --warmup 100 --no-cpu-baseline --no-single-ply --no-masked >> $OUT/sweep.jsonl
echo done
