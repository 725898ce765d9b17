# round 6, batch i: the play kernels' fixed cost per launch against plies per launch (tools/probe_plies.py under a kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o plies -- python3 $R/tools/probe_plies.py > $O/probe.log 2>&1 || exit 1
cd $R && python3 tools/probe_plies.py --trace "$O/trace/**/plies_results.db" > $O/plies.json && cat $O/plies.json
