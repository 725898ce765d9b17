# Round 4, batch h: the suite and smoke on the kept form (random play resets a
# full board before the scan, greedy in the terminal block), greedy against the
# all-terminal-block build (oldterm), and the bench.
set -o pipefail
O=${1:-gpurun_out/r04h}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in "greedy 8 100 10" "greedy 8 10 10" "random 8 100 0"; do
  set -- $cfg
  timeout -k 10 300 python tools/ab_variants.py --run new oldterm --policy $1 --board-size $2 --plies $3 --init-rand $4 --launches 10 >> $O/ab_term.jsonl 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab_term.jsonl
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
head -c 400 $O/bench.json
