# A/B: legal_moves (Solo engine: k_step, k_sample_step, ...) on dwords for multi-word boards (OTH_DW_LEGAL)
set -o pipefail
O=${1:-gpurun_out/r02dwl}; mkdir -p $O
for n in 10 12 16; do
timeout -k 10 300 python tools/ab_sample_step.py dwl0 dwl1 --board-size $n > $O/ss_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ss_n$n.json
done
for n in 10 16; do
timeout -k 10 300 python tools/ab_step.py dwl0 dwl1 --board-size $n > $O/step_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/step_n$n.json
done
