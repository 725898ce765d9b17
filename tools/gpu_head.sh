# GPU validation of HEAD: full gpu suite, smoke, then the round-end measurements
set -o pipefail
O=${1:-gpurun_out/r02head}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
cat $O/smoke.log
bash tools/gpu_final.sh $O
