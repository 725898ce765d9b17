# A/B of k_play_rand changes (variants built by tools/ab_variants.py --build):
# v0 = round-start code (OTH_SELECT_LDS=0 OTH_TALLY_SIGN=0 OTH_PHILOX_XOR3=0),
# v1 = all on, v2 = without the LDS select table.  Then the GPU suite on the main build.
set -o pipefail
O=${1:-gpurun_out/r03d}; shift; V="${*:-v0 v1 v2}"; mkdir -p $O
export TMPDIR=/tmp
for spec0 in "random 0 8 100 65536" "random 0 6 100 65536" "greedy 10 8 10 65536" "random 0 8 100 131072"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run $V --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
