# packed meta / dones stores in the single-ply kernels: q0 per-lane 2-byte / 1-byte stores,
# q1 a lane pair's meta and a lane quad's dones as one dword; then the GPU suite on the main build
set -o pipefail
O=${1:-gpurun_out/r03n}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_ply.py q0 q1 --envs 65536,262144,1048576 --rounds 8 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
