set -o pipefail
O=gpurun_out/r02zb; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_masked.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python tools/ab_sample_step.py b0 a1 a2 a3 --no-check > $O/abl.json 2> $O/abl.err || { tail -20 $O/abl.err; exit 1; }
cat $O/abl.json
timeout -k 10 240 python tools/ab_sample_step.py b0 a1 a2 a3 --no-check --envs 16384 > $O/abl16k.json 2> $O/abl.err || { tail -20 $O/abl.err; exit 1; }
cat $O/abl16k.json
