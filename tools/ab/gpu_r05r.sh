# round 5, batch r: the learners' ply with its make_state in producer / consumer
# blocks (ssopc2: 4 producer waves sampling and stepping two groups of 32 boards
# in turn, 4 consumer waves streaming the previous group's observation) against
# k_sample_step2 + its tail (head)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssopc2 --envs 65536 > $O/ab_ss_obs_65k.json 2> $O/ab_ss_obs_65k.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssopc2 --envs 65536 --layout board --dtype int64 > $O/ab_ss_obs_65k_board.json 2> $O/ab_ss_obs_65k_board.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssopc2 --envs 131072 > $O/ab_ss_obs_131k.json 2> $O/ab_ss_obs_131k.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssopc2 --envs 70001 > $O/ab_ss_obs_70k.json 2> $O/ab_ss_obs_70k.err || exit 1
echo batch-r-done
