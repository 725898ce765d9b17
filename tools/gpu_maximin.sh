#!/bin/bash
# GPU check of MaxiMin's planes-based last level: parity suite, then A/B
# (variants: tools/ab_variants.py --build base= mp0=-DOTH_MAXIMIN_PLANES=0)
set -e
O=${1:-gpurun_out/maximin}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
: > $O/ab.jsonl
for pol in maximin2 maximin3; do
  for n in 6 8 10; do
    timeout -k 10 150 python tools/ab_variants.py --run base mp0 --board-size $n --plies 4 --launches 5 --rounds 4 --policy $pol --init-rand 6 --envs 16384 >> $O/ab.jsonl 2>>$O/ab.err
  done
done
echo ok
