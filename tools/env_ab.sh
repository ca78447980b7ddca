#!/bin/bash
# Generic environment-switch A/B of a bench leg (through gpurun, from the repo root):
#   bash tools/env_ab.sh OUTDIR "A=1,B=2" "A=0" ...   -- each config (comma-separated VAR=value
# pairs, "-" for none) runs the bench, PASSES (default 2) rounds over the list.  Default: the
# 10-step C2 leg alone; AB_ARGS replaces the bench arguments (e.g. a stacked-pairs leg).
# Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
ARGS=${AB_ARGS:-"--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 10"}
for pass in $(seq 1 ${PASSES:-2}); do
  for cfg in "$@"; do
    envs=()
    [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 ${AB_TIMEOUT:-150} python3 bench.py $ARGS --detail-json "" | sed "s|^|$cfg |" >> $O/bench.txt
  done
done
echo done
