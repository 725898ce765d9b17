# round 6, batch a: greedy run lengths by window doubling (head, OTH_GREEDY_DBL=1)
# against the nested thermometer (g0, OTH_GREEDY_DBL=0), config 3 at 65,536
# boards (10- and 100-ply launches, 0-10-ply openings); the new GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_distributed.py tests/test_gpu_hazards.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head g0 --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head g0 --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head g0 --policy greedy --plies 100 --init-rand 0 > $O/greedy100_noopen.json 2> $O/greedy100_noopen.err || exit 1
echo batch-a-done
