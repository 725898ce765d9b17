# round 5, batch g: the whole GPU suite and smoke after removing the A/B-only
# switches and the rejected greedy-pair kernel; MaxiMin (depth 2-4, 65,536 8x8
# boards) kernel trace and counters
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=10 tests -m gpu > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/prof_maximin.py > $O/maximin_times.jsonl 2> $O/maximin.err || exit 1
export TMPDIR=/tmp
cd /tmp
D=$O/maximin
mkdir -p $D
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/prof_maximin.py > $D/trace.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $D/pmc$i -o run -- python3 $R/tools/prof_maximin.py > $D/pmc$i.log 2>&1 || exit 1
done
python3 $R/tools/kstats.py $D --match maximin --json $D/kstats.json > /dev/null || exit 1
echo batch-g-done
