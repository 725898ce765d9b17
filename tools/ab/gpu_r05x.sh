# round 5, batch x: config 1 (one board through the drop-in OthelloEnv against
# RandomPolicy) -- the whole step, the bare oth_step_sync call, a cProfile of the
# loop, and the kernel trace of the same run
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_config1.py > $O/prof_config1.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/prof_config1.py --seconds 0.3 > $O/trace.log 2>&1 || exit 1
echo batch-x-done
