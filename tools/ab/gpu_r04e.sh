# Round 4, batch e: block size of the single-ply kernels (256 / 128 / 64 threads,
# and 64 with computed rays at every size) at 65,536 and 1,048,576 boards.
set -o pipefail
O=${1:-gpurun_out/r04e}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "single_ply or external" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/ab_ply.py new b128 b64 b64m --envs 65536,1048576 --rounds 8 > $O/ab_block.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_block.jsonl
