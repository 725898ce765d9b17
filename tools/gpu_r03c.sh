# GPU tests of the size-selected single-ply kernels, then the graph-replayed paths' kernel trace
set -o pipefail
O=${1:-gpurun_out/r03c}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hazards.py -q -x --timeout 300 --timeout-method thread -k "ray_sources or external or live or split or golden or kat" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/prof_step.py --envs 65536,1048576 --cases step_ext,play1,sample_step,sample_only,sample_then_step > $O/times.jsonl 2> $O/times.err || { tail $O/times.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/prof_step.py --envs 65536,1048576 --cases step_ext,play1,sample_step,sample_only,sample_then_step > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep -v '"rep": 0' $O/times.jsonl
