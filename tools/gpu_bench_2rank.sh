# bench.py's multi-rank path at HEAD on one GPU: 2 gloo ranks vs 1 rank at the same 131,072 global boards (W/D/L must agree)
set -o pipefail
O=${1:-gpurun_out/r02rank}; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --global-envs 131072 --steps 10 --warmup 2 --no-cpu-baseline --no-side > $O/bench_1rank.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
OTH_BENCH_BACKEND=gloo OTH_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --global-envs 131072 --steps 10 --warmup 2 --no-cpu-baseline --no-side > $O/bench_2rank.json 2> $O/b2.err || { tail $O/b2.err; exit 1; }
python -c "
import json
a=json.loads(open('$O/bench_1rank.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/bench_2rank.json').read().strip().splitlines()[-1])
print('1 rank', a['value'], a['wdl']); print('2 ranks', b['value'], b['wdl'], b['n_gpus'])
assert a['wdl']==b['wdl'], 'W/D/L differ'
print('W/D/L identical')
"
