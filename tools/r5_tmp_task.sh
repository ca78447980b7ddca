set -e -o pipefail
O=gpurun_out/r5f; mkdir -p $O
AESFHE_BOOT_LOW=0 AESFHE_NTT_INV8=0 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_inv16.json
AESFHE_BOOT_LOW=0 AESFHE_NTT_INV8=1 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_inv8.json
AESFHE_BOOT_LOW=0 AESFHE_NTT_FWD8=1 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_fwd8.json
cat $O/digest_inv16.json $O/digest_inv8.json $O/digest_fwd8.json
PASSES=1 bash tools/env_ab.sh r5f AESFHE_NTT_INV8=0,AESFHE_BOOT_LOW=0 AESFHE_NTT_INV8=1,AESFHE_BOOT_LOW=0 AESFHE_NTT_INV8=1,AESFHE_NTT_FWD8=1,AESFHE_BOOT_LOW=0 AESFHE_BOOT_LOW=1
python3 - <<'PY'
import json
for l in open('gpurun_out/r5f/bench.txt'):
    cfg, js = l.split(' ', 1); d = json.loads(js); c = d['roofline_step']['classes']
    print(cfg, d["value"], d["launches_per_encrypt"], d["precision"]["margin_factor"], 'rows_inv', c['ntt_rows_inv'][:3], 'rows_fwd', c['ntt_rows_fwd'][:3], 'key_inner', c['key_inner'][:3])
PY
rc=0; timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boot_low.py -m gpu -v -s --timeout 250 --timeout-method thread > $O/pytest_low.log 2>&1 || rc=$?
tail -15 $O/pytest_low.log
[ $rc -le 1 ] || exit $rc
rc=0; timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || rc=$?
tail -12 $O/pytest_all.log
# test failures (rc 1) are reported and the measurements go on; a crash / time limit ends the call
[ $rc -le 1 ] || exit $rc
bash tools/gpu_task.sh r5f pmcbench
python3 -c "
import json; d=json.load(open('gpurun_out/r5f/pmc_traffic_bench.json')); print({k: (round(v.get('traffic_over_algorithmic') or 0,3)) for k,v in d.items() if isinstance(v, dict) and 'traffic_over_algorithmic' in v})"
bash tools/sq_pmc.sh r5f/sq_c2
SQ_ARGS="pairs=16" bash tools/sq_pmc.sh r5f/sq_pairs16
