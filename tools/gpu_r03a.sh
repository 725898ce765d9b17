# round-3 validation: new single-ply kernels, hazards, full GPU suite, then timings + kernel trace
set -o pipefail
O=${1:-gpurun_out/r03a}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hazards.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "external or hazards or live or u2 or kat or golden or split" > $O/pytest_quick.log 2>&1 || { echo QUICK_FAIL; tail -40 $O/pytest_quick.log; exit 1; }
tail -2 $O/pytest_quick.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_prof_step.sh $O/step "--plies 32" > $O/step.log 2>&1 || { tail $O/step.log; exit 1; }
cat $O/step/times.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 4 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
