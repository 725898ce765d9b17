# single-ply launches above 65,536 boards: n0 plain stores, n1 nontemporal stores (OTH_PLY_NT)
set -o pipefail
O=${1:-gpurun_out/r03l}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/ab_ply.py n0 n1 --envs 262144,1048576 --rounds 8 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
