set -e -o pipefail
O=gpurun_out/r5g; mkdir -p $O
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boot_low.py -m gpu -v -s --timeout 250 --timeout-method thread > $O/pytest_low.log 2>&1 || rc=$?
grep -E "PASSED|FAILED|err|margin| [0-9.]+ enc" $O/pytest_low.log | head -20
[ $rc -eq 0 ] || { tail -30 $O/pytest_low.log; exit 1; }
PASSES=1 bash tools/env_ab.sh r5g AESFHE_BOOT_LOW=0 AESFHE_BOOT_LOW=1
python3 - <<'PY'
import json
for l in open('gpurun_out/r5g/bench.txt'):
    cfg, js = l.split(' ', 1); d = json.loads(js); c = d['roofline_step']['classes']
    print(cfg, d["value"], d["launches_per_encrypt"], d["precision"]["margin_factor"], d["precision"]["worst_stage"], 'rows_fwd', c['ntt_rows_fwd'][:3], 'key_inner', c['key_inner'][:3])
PY
rc=0; timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || rc=$?
tail -12 $O/pytest_all.log
[ $rc -le 1 ] || exit $rc
bash tools/sq_pmc.sh r5g/sq_c2
SQ_ARGS="pairs=16" bash tools/sq_pmc.sh r5g/sq_pairs16
bash tools/gpu_task.sh r5g pmcbench
