set -e -o pipefail
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_deferred_calls.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_def.log 2>&1 || { tail -40 $O/pytest_def.log; exit 1; }
tail -3 $O/pytest_def.log
timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 1 --detail-json $O/detail.json > $O/bench.json 2> $O/bench.err
bash tools/r5_ki8_task.sh
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { tail -40 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
