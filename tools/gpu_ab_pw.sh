# A/B: oth_sample_step on lane pairs for two-word boards (OTH_SS_PAIR_W) vs one lane per board
set -o pipefail
O=${1:-gpurun_out/r02pw}; mkdir -p $O
for args in "--board-size 10" "--board-size 10 --lp" "--board-size 9" "--board-size 11" "--board-size 10 --envs 16384" "--board-size 10 --envs 777"; do
tag=$(echo "$args" | tr -d ' -')
timeout -k 10 300 python tools/ab_sample_step.py pw0 pw1 $args > $O/ss_$tag.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ss_$tag.json
done
