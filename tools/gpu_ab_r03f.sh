# The GPU suite on the main build, then A/B of boards per lane in the big single-ply
# launches (k1 / k2 / k4 = OTH_PLY_K_BIG 1 / 2 / 4, N = 8 variants) and the fused ply
# of the current tree (k1) at the pair and quad sizes.
set -o pipefail
O=${1:-gpurun_out/r03f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python -u tools/ab_ply.py k1 k2 k4 --envs 262144,1048576 --rounds 6 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
for E in 65536 16384; do
timeout -k 10 240 python -u tools/ab_sample_step.py k1 --envs $E --board-size 8 > $O/ss_n8_$E.json 2> $O/ab_ss_$E.err || { tail -20 $O/ab_ss_$E.err; exit 1; }
cat $O/ss_n8_$E.json
done
# multi-word random play (10x10): w0 = without the LDS select table and the sign tally, w1 = with
timeout -k 10 300 python tools/ab_variants.py --run w0 w1 --plies 100 --launches 10 --rounds 8 --policy random --board-size 10 --envs 65536 > $O/ab_random_10_65536.json 2> $O/ab_w.err || { tail -20 $O/ab_w.err; exit 1; }
cat $O/ab_random_10_65536.json
