# A/B of the single-ply kernel variants (tools/ab_ply.py), built beforehand by tools/ab_variants.py --build
set -o pipefail
O=${1:-gpurun_out/abply}; shift; mkdir -p $O
timeout -k 10 600 python tools/ab_ply.py "$@" > $O/ab.jsonl 2> $O/ab.err || { tail -30 $O/ab.err; exit 1; }
cat $O/ab.jsonl
