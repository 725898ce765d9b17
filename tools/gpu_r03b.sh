# round-3 validation 2: full GPU suite, smoke, kernel trace + counters of the single-ply paths, bench
set -o pipefail
O=${1:-gpurun_out/r03b}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_prof_step.sh $O/step "--plies 32" > $O/step.log 2>&1 || { tail $O/step.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
