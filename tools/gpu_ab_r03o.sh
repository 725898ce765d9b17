# k_sample_step2's flips split over the lane pair (f1, RAYS_PAIR) against both lanes computing all
# eight directions (f0); then the GPU suite on the main build
set -o pipefail
O=${1:-gpurun_out/r03o}; mkdir -p $O
export TMPDIR=/tmp
for E in 65536 32768; do
timeout -k 10 240 python -u tools/ab_sample_step.py f0 f1 --envs $E > $O/ab_ss_$E.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_ss_$E.json
done
timeout -k 10 240 python -u tools/ab_sample_step.py f0 f1 --envs 65536 --board-size 7 > $O/ab_ss7_65536.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_ss7_65536.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
