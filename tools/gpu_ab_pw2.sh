# A/B: two-word lane pairs at latency-bound sizes for boards whose rows are not float4-aligned (9x9, 11x11)
set -o pipefail
O=${1:-gpurun_out/r02pw2}; mkdir -p $O
for args in "--board-size 9 --envs 16384" "--board-size 11 --envs 16384" "--board-size 9 --envs 32768" "--board-size 11 --envs 4096" "--board-size 10 --envs 32768"; do
tag=$(echo "$args" | tr -d ' -')
timeout -k 10 300 python tools/ab_sample_step.py pw0 pw1 $args > $O/ss_$tag.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ss_$tag.json
done
