set -e
mkdir -p gpurun_out/sweep
for E in 65536 131072 262144; do
  for P in 1 10 50 200; do
    timeout -k 10 120 python bench.py --envs $E --plies-per-launch $P --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/sweep/E${E}_P${P}.json 2>/dev/null
  done
done
timeout -k 10 120 python bench.py --envs 65536 --plies-per-launch 50 --steps 2000 --no-record --no-cpu-baseline > gpurun_out/sweep/norecord.json 2>/dev/null
timeout -k 10 300 python bench.py --policy greedy --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/sweep/greedy.json 2>/dev/null
for n in 6 10 16; do timeout -k 10 120 python bench.py --board-size $n --steps 1000 --no-cpu-baseline > gpurun_out/sweep/N$n.json 2>/dev/null; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01 -o run -- python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
