#!/bin/bash
# A/B of one environment switch on the C2 headline leg, interleaved on one box: VAR=0 / default,
# three times each; GPU tests given run first.  usage: [OFF=value] bash tools/r3_ab.sh OUT VAR [tests...]
# (the "off" leg sets VAR=$OFF, default 0)
set -e -o pipefail
O=gpurun_out/${1:-r3ab}
VAR=$2
shift 2 || true
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --steps 10 --warmup 2"
if [ $# -gt 0 ]; then
    timeout -k 10 900 python3 -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
fi
for i in 1 2 3; do
    env $VAR=${OFF:-0} timeout -k 10 300 python3 bench.py $B > $O/bench_off_$i.json
    timeout -k 10 300 python3 bench.py $B > $O/bench_on_$i.json
done
echo done
