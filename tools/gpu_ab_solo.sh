set -o pipefail
O=gpurun_out/r02zc; mkdir -p $O
run() { local out=$1; shift; timeout -k 10 240 python tools/ab_sample_step.py "$@" > $O/$out.json 2> $O/$out.err || { tail -20 $O/$out.err; exit 1; }; echo "$out"; cat $O/$out.json; }
run solo_n8 d0 so
run solo_n8_lp d0 so --lp
run solo_n7_lp d0 so --lp --board-size 7
run solo_abl d0 so so1 --no-check
