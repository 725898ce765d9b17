# round 5, batch l: oth_observe against torch's fill_ of the same tensor at
# 1,048,576 boards with 4 / 8 / 16 boards per wave (64 shipped), and the pure
# store stream (cst: no board words fetched, other values) at 65,536 and 1,048,576
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_observe.py head bpw4 bpw8 bpw16 --envs 1048576 --launches 20 --rounds 4 > $O/ab_obs_bpw.jsonl 2> $O/ab_obs_bpw.err || exit 1
timeout -k 10 300 python -u tools/ab_observe.py head cst --no-check --envs 65536,1048576 --launches 20 --rounds 4 > $O/ab_obs_cst.jsonl 2> $O/ab_obs_cst.err || exit 1
echo batch-l-done
