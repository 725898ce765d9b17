set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
OTH_BENCH_DEVICE=0 OTH_BENCH_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank_gloo.json 2> $O/bench_2rank.err || exit 1
OTH_BENCH_DEVICE=0 OTH_BENCH_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --global-envs 131072 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank_g131072.json 2>> $O/bench_2rank.err || exit 1
timeout -k 10 200 python bench.py --envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-side > $O/bench_1rank_g131072.json 2>> $O/bench_2rank.err || exit 1
bash tools/pmc_profile.sh $O/pmc > $O/pmc.log 2>&1 || exit 1
echo ALLOK
