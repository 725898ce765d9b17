# round 5, batch c: the learners' fused ply with make_state on lane quads
# (variant ssoq) against lane pairs; random 10x10 play at 65,536 and 131,072
# boards (one and two waves per SIMD: the issue gain a lane-pair split would
# have to beat) with counters; the bench with the compact line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssoq > $O/ab_ss_obs.json 2> $O/ab_ss_obs.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssoq --envs 32768 > $O/ab_ss_obs_32768.json 2>> $O/ab_ss_obs.err || exit 1
for E in 65536 131072; do
  timeout -k 10 200 python -u tools/ab_variants.py --run head --board-size 10 --envs $E --plies 100 --launches 10 > $O/rand10_$E.json 2>> $O/rand10.err || exit 1
done
export TMPDIR=/tmp
cd /tmp
for E in 65536 131072; do
  D=$O/rand10_prof_$E
  mkdir -p $D
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/ab_variants.py --run head --board-size 10 --envs $E --plies 100 --launches 5 --rounds 1 > $D/trace.log 2>&1 || exit 1
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 $R/tools/ab_variants.py --run head --board-size 10 --envs $E --plies 100 --launches 5 --rounds 1 > $D/pmc$i.log 2>&1 || exit 1
  done
  python3 $R/tools/kstats.py $D --match k_play --json $D/kstats.json > /dev/null || exit 1
done
cd $R
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo batch-c-done
