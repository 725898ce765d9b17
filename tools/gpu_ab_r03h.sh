# The GPU suite on the main build; A/B of the current tree (cur) against the last
# commit (base, built from a git worktree for N = 8): k_play_rand with alternating word
# roles and buffer-descriptor stores, single plies with the half ray table; the default bench.
set -o pipefail
O=${1:-gpurun_out/r03h2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for spec0 in "random 0 8 100 65536" "random 0 6 100 65536" "greedy 10 8 10 65536" "random 0 8 100 131072" "random 0 7 100 65536"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run base cur --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
timeout -k 10 240 python -u tools/ab_ply.py base cur --envs 65536,262144,1048576 --rounds 6 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
