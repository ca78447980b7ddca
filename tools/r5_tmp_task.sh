set -e -o pipefail
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boot_chunk.py tests/test_gpu_deferred_calls.py tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
tail -2 $O/pytest_a.log
for v in 0 1 0 1; do AESFHE_LIN_MAC_NB4=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 64 --pair-stack 64 --pair-steps 1 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --detail-json $O/pairs_nb4_$v.json > /dev/null 2> $O/pairs.err; python3 -c "
import json; d=json.load(open('$O/pairs_nb4_$v.json'))['batch_pairs']; c=d['roofline_step']['classes']
print('nb4=$v', round(d['blocks_per_s'],3), round(d['ms_per_pair'],2), {k: (round(v['frac'],3), round(v['avg_us'],1)) for k, v in c.items()})" | tee -a $O/pairs_ab.txt; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { tail -40 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
