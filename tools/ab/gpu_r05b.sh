# round 5, batch b: the whole GPU suite and smoke on the fused-step default (lane
# pairs), the sample-step observation tail's cost when unused (variant ssnoobs),
# MaxiMin on a wave per board against one lane per board (variant mmlane), the
# bench, the headline's kernel trace, counters of greedy play on lane pairs
# (variant gp1) against k_play_rand<8, GREEDY>, and the sustained clock
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_sample_step.py head ssnoobs --lp > $O/ab_ss_tail.json 2> $O/ab_ss_tail.err || exit 1
timeout -k 10 300 python -u tools/ab_maximin.py mmlane > $O/ab_maximin.jsonl 2> $O/ab_maximin.err || exit 1
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-side --no-cpu-baseline --steps 20 --warmup 5 > $O/trace.log 2>&1 || exit 1
for nm in head gp1; do
  D=$O/greedy_$nm
  mkdir -p $D
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/ab_variants.py --run $nm --policy greedy --init-rand 10 --plies 100 --launches 5 --rounds 1 > $D/trace.log 2>&1 || exit 1
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 $R/tools/ab_variants.py --run $nm --policy greedy --init-rand 10 --plies 100 --launches 5 --rounds 1 > $D/pmc$i.log 2>&1 || exit 1
  done
  python3 $R/tools/kstats.py $D --match k_play --json $D/kstats.json > /dev/null || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/clk -o run -- python3 $R/tools/sustained_clock.py --plies 1000 --seconds 3 > $O/clk.log 2>&1 || exit 1
python3 $R/tools/sustained_clock.py --summarize $O/clk > $O/clk.json || exit 1
timeout -k 10 60 python3 $R/tools/sustained_clock.py --plies 100 --seconds 3 > $O/sustained100.json 2>&1 || exit 1
echo batch-b-done
