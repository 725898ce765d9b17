#!/bin/bash
# rocprofv3 counter passes for the bench kernel (run on the GPU box).
# Usage: bash tools/pmc_profile.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:-"--steps 50 --warmup 5 --no-cpu-baseline --no-side"}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
done
echo done
