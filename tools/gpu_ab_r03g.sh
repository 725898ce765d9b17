# The GPU suite on the main build, then the single-ply ray source above 65,536 boards:
# h0 = the whole table in LDS (16 B per thread), h1 = its four up directions (8 B per thread)
set -o pipefail
O=${1:-gpurun_out/r03g}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python -u tools/ab_ply.py h0 h1 --envs 262144,1048576 --rounds 8 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
