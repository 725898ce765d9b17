# round 5, batch u: traces and counters of the fused step / learner ply with
# their observations, one case per run so each kernel's counters belong to one
# layout (65,536 8x8 boards)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
export TMPDIR=/tmp
for c in step_obs step_obs_ms ss_obs; do
  bash tools/gpu_prof_step.sh $O/$c --envs 65536 --plies 32 --cases $c > $O/$c.log 2>&1 || { tail $O/$c.log; exit 1; }
  python3 tools/kstats.py $O/$c --json $O/$c/kstats.json > /dev/null || exit 1
done
echo batch-u-done
