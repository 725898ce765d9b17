#!/bin/bash
# GPU check of the multi-word greedy planes: parity suite, then A/B against the
# candidate loop (variants built by tools/ab_variants.py --build base= pw0=-DOTH_GREEDY_PLANES_W=0)
set -e
O=${1:-gpurun_out/planes_w}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
: > $O/ab.jsonl
for n in 10 12 16; do
  timeout -k 10 150 python tools/ab_variants.py --run base pw0 --board-size $n --plies 10 --launches 10 --rounds 6 --policy greedy --init-rand 6 >> $O/ab.jsonl 2>>$O/ab.err
done
timeout -k 10 150 python tools/ab_step.py base pw0 --board-size 10 >> $O/ab.jsonl 2>>$O/ab.err
echo ok
