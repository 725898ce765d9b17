set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
for spec in "random 0 8" "random 10 8" "random 0 6" "random 0 7" "random 0 4"; do
set -- $spec
timeout -k 10 300 python tools/ab_variants.py --run pp0 pp1 --plies 100 --launches 10 --rounds 6 --policy $1 --init-rand $2 --board-size $3 > $O/ab_$1_$2_$3.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec"; cat $O/ab_$1_$2_$3.json
done
