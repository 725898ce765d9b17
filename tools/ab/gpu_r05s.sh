# round 5, batch s: oth_observe's large-launch shapes over sizes -- 4-KiB output
# regions (the head build of the time), 64 boards a wave (reg64k), 16-KiB regions
# (reg16k), 64 boards a wave in strided 4-KiB chunks (chunk: a probe since
# removed, OTH_OBS_CHUNK) -- with torch's fill_ of the same tensors; variants:
#   python tools/ab_variants.py --sizes 8 --build reg64k=-DOTH_OBS_LARGE_REGION=65536 \
#       reg16k=-DOTH_OBS_LARGE_REGION=16384 chunk=-DOTH_OBS_CHUNK=1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_observe.py head chunk --envs 1048576,262144 --launches 20 --rounds 4 > $O/ab_obs_chunk.jsonl 2> $O/ab_obs_chunk.err || exit 1
timeout -k 10 600 python -u tools/ab_observe.py head reg64k reg16k chunk --envs 262144,524288,1048576,2097152 --launches 10 --rounds 4 > $O/ab_obs_sweep.jsonl 2> $O/ab_obs_sweep.err || exit 1
echo batch-s-done
