# Round 4, batch f: two boards per lane for large oth_step launches (the second
# board's loads in flight while the first is stepped and stored).
set -o pipefail
O=${1:-gpurun_out/r04f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "single_ply or external or random_rollout" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/ab_ply.py new bpl2 --envs 262144,1048576 --rounds 8 > $O/ab_bpl2.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_bpl2.jsonl
