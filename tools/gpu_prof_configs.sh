# Kernel traces + counter passes of BASELINE configs 3 / 5 and the observation
# encoders (tools/prof_configs.py), one output directory per case group.
# Usage: bash tools/gpu_prof_configs.sh <outdir> [case groups, e.g. greedy10 greedy100 rand6,rand10 obs]
set -o pipefail
O=${1:-gpurun_out/r04cfg}; shift || true
CASES=${@:-"greedy10 greedy100 rand6,rand10 obs"}
export TMPDIR=/tmp
for G in $CASES; do
  D=$O/$(echo $G | tr ',' '_')
  mkdir -p $D
  timeout -k 10 200 python3 tools/prof_configs.py --cases $G > $D/times.jsonl 2> $D/times.err || { tail $D/times.err; exit 1; }
  cat $D/times.jsonl
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/prof_configs.py --cases $G > $D/trace.log 2>&1 || { tail $D/trace.log; exit 1; }
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 tools/prof_configs.py --cases $G --launches 5 > $D/pmc$i.log 2>&1 || { tail $D/pmc$i.log; exit 1; }
  done
  python3 tools/kstats.py $D --json $D/kstats.json > /dev/null || exit 1
done
echo done
