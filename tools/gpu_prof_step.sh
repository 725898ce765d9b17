# Kernel trace + counter passes of the single-ply paths (tools/prof_step.py) at
# 65,536 and 1,048,576 8x8 boards.  Usage: bash tools/gpu_prof_step.sh <outdir> [prof_step args]
set -o pipefail
O=${1:-gpurun_out/r03step}; shift || true
ARGS=${@:-"--plies 32"}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prof_step.py $ARGS > $O/times.jsonl 2> $O/times.err || { tail $O/times.err; exit 1; }
cat $O/times.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/prof_step.py $ARGS > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 tools/prof_step.py $ARGS > $O/pmc$i.log 2>&1 || { tail $O/pmc$i.log; exit 1; }
done
echo done
