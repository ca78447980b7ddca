set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
C2="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 10 --detail-json ''"
for pass in 1 2; do
  for cfg in "17 5" "9 5" "9 4" "9 3" "9 2"; do
    set -- $cfg
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 \
        --eager-steps 0 --deferred-steps 0 --steps 10 --detail-json "" --fresh-level $1 --dnum $2 | sed "s|^|L$1_d$2 |" >> $O/bench.txt
  done
done
echo done
