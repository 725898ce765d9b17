# nontemporal-store probes: p0 defaults (large single-ply launches nontemporal), p1 small single-ply
# launches too, p2 k_play_rand's per-ply outputs; then the GPU suite on the main build
set -o pipefail
O=${1:-gpurun_out/r03m}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/ab_ply.py p0 p1 --envs 65536,1048576 --rounds 8 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
for spec0 in "random 0 8 100 65536" "random 0 8 100 131072"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run p0 p2 --plies $4 --launches 10 --rounds 10 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
