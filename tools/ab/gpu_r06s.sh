# round 6, batch s: where the play kernels' waiting cycles go -- branch, instruction
# fetch, LDS and VMEM-store counters of config 3 (greedy100), config 2 (rand8) and
# 10x10 (rand10), one counter set per pass (tools/prof_configs.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s
mkdir -p $O
cd $R
export TMPDIR=/tmp
for G in greedy100 rand8 rand10; do
  D=$O/$G
  mkdir -p $D
  i=0
  for set in "SQ_WAVES SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
             "SQ_WAVES SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_ANY" \
             "SQ_WAVES SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 tools/prof_configs.py --cases $G --launches 5 > $D/pmc$i.log 2>&1 || { tail $D/pmc$i.log; exit 1; }
  done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/prof_configs.py --cases $G --launches 5 > $D/trace.log 2>&1 || { tail $D/trace.log; exit 1; }
  python3 tools/kstats.py $D --json $D/kstats.json > /dev/null || exit 1
done
echo batch-s-done
