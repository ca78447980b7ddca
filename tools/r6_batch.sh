set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
C2="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
PB="--steps 1 --warmup 1 $C2 --detail-json $O/pmcf_detail.json --whole-stats $O/ws_unused.json"
HIP_ENABLE_DEFERRED_LOADING=0 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcb_fetch -o run -- python3 bench.py $PB > $O/pmcb_fetch.out 2> $O/pmcb_fetch.err
echo done
