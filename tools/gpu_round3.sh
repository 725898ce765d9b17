set -o pipefail
O=${1:-gpurun_out/r02n}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/pmc_profile.sh $O/pmc > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
echo pmc done
