# round-end measurements: default + driver-shaped bench, PMC passes, fused-path graph benches
set -o pipefail
O=${1:-gpurun_out/r02final}; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail $O/bench_driver.err; exit 1; }
tail -1 $O/bench_driver.json
bash tools/pmc_profile.sh $O/pmc > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
for a in "--fused" "--fused --device-draws" "--fused --board-size 6" "--fused --board-size 10" "--fused --envs 16384" "--fused --envs 4096" "--fused --board-size 6 --envs 4096"; do
timeout -k 10 200 python tools/bench_graph.py $a >> $O/graph.jsonl 2> $O/graph.err || { tail $O/graph.err; exit 1; }
done
cat $O/graph.jsonl
