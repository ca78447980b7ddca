set -e -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_flag_identity.py" bash tools/gpu_task.sh r6e tests
PASSES=2 bash tools/env_ab.sh r6e "-" "AESFHE_KI8_OCC=4" "AESFHE_RENORM_FOLDS=1"
AB_TIMEOUT=200 PASSES=1 AB_ARGS="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 64 --pair-stack 64 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 2 --warmup 1" bash tools/env_ab.sh r6e_stack "-" "AESFHE_KI8_OCC=4"
bash tools/gpu_task.sh r6e pmcbench
O=gpurun_out/r6e
C2="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ctl_fetch -o run -- python3 bench.py --steps 1 --warmup 1 $C2 --detail-json "" --whole-stats $O/ws_ctl.json > $O/ctl_fetch.out 2> $O/ctl_fetch.err || echo "control rc=$?" > $O/ctl_rc.txt
rm -rf $O/ctl_fetch
echo done
