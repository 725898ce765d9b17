#!/bin/bash
# rocprofv3 kernel trace + HBM counter passes for the masked-categorical kernel
# (run on the GPU box).  Usage: bash tools/masked_profile.sh <outdir>
set -e
OUT=${1:-gpurun_out/masked_prof}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--envs 4194304 --iters 20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_masked.py $ARGS > $OUT/trace.log 2>&1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 tools/bench_masked.py $ARGS > $OUT/pmc$i.log 2>&1
done
echo done
