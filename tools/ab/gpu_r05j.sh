# round 5, batch j: the whole GPU suite after 8-byte observations by pairs of
# squares (OTH_OBS_PAIR8) and MaxiMin's nested subtrees below
# OTH_MM_NESTED_MAX_E boards; A/B against quad stores (quad8) at 65,536 and
# 1,048,576 boards, and the MaxiMin threshold (mmnest: always nested, mmflat: never)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants quad8 > $O/ab_step_obs.json 2> $O/ab_step_obs.err || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants quad8 --envs 1048576 --plies 8 --rounds 4 > $O/ab_step_obs_1m.json 2> $O/ab_step_obs_1m.err || exit 1
timeout -k 10 400 python -u tools/ab_maximin.py mmnest --envs 16384 4096 2048 1024 --depths 4 5 > $O/ab_mm_nest.jsonl 2> $O/ab_mm_nest.err || exit 1
timeout -k 10 400 python -u tools/ab_maximin.py mmflat --envs 16384 4096 2048 1024 --depths 4 5 > $O/ab_mm_flat.jsonl 2> $O/ab_mm_flat.err || exit 1
echo batch-j-done
