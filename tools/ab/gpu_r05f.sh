# round 5, batch f: counters of k_play_rand<8, random> at 65,536 (one wave per
# SIMD) and 131,072 boards (two waves: config 4's per-GPU shard) -- where the
# second wave's issue time goes (instruction-issue waits against data waits)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for E in 65536 131072; do
  D=$O/rand8_$E
  mkdir -p $D
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/ab_variants.py --run head --board-size 8 --envs $E --plies 100 --launches 5 --rounds 1 > $D/trace.log 2>&1 || exit 1
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 $R/tools/ab_variants.py --run head --board-size 8 --envs $E --plies 100 --launches 5 --rounds 1 > $D/pmc$i.log 2>&1 || exit 1
  done
  python3 $R/tools/kstats.py $D --match k_play --json $D/kstats.json > /dev/null || exit 1
done
echo batch-f-done
