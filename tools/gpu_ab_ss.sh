set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
run() { local out=$1; shift; timeout -k 10 240 python tools/ab_sample_step.py "$@" > $O/$out.json 2> $O/$out.err || { tail -20 $O/$out.err; exit 1; }; echo "$out"; cat $O/$out.json; }
run mx_n8 mx0 mx1
run mx_n8_lp mx0 mx1 --lp
run mx_n6 mx0 mx1 --board-size 6
run abl_n8 mx1 abl1 abl2 --no-check
run abl_n8_lp mx1 abl1 abl2 --no-check --lp
timeout -k 10 600 python -u -m pytest tests/test_gpu_masked.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
