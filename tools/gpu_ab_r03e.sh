# A/B (N = 8 variants, tools/ab_variants.py --sizes 8 --build):
#  fused sample + step: s0 Duo (default), s1 step1 with LDS rays, s2 step1 with computed rays,
#  s3 = s2 + per-wave W/D/L slots;  single ply: c0 cap test without bitop3, m1 computed rays at every size
set -o pipefail
O=${1:-gpurun_out/r03e}; mkdir -p $O
export TMPDIR=/tmp
for E in 65536 16384; do
timeout -k 10 240 python -u tools/ab_sample_step.py s0 s1 s2 s3 --envs $E --board-size 8 > $O/ss_n8_$E.json 2> $O/ab_ss_$E.err || { tail -20 $O/ab_ss_$E.err; exit 1; }
cat $O/ss_n8_$E.json
done
timeout -k 10 240 python -u tools/ab_ply.py c0 s0 m1 --envs 65536,1048576 --rounds 6 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail -20 $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
