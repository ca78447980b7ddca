set -e -o pipefail
O=gpurun_out/${1:-r5x}; mkdir -p $O
PASSES=2 bash tools/env_ab.sh ${1:-r5x} AESFHE_SB_NIB=0 -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    print(cfg, 'C2', d['value'], 'launches', d['launches_per_encrypt'], 'precision', d['precision']['margin_factor'], d['precision']['max_err_rad'], d['precision']['worst_stage'])
PY
for v in 0 1; do
  AESFHE_SB_NIB=$v timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch-states 1024 --batch-steps 2 \
      --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --detail-json '' > $O/nib_$v.json
  python3 -c "
import json; d=json.loads(open('$O/nib_$v.json').read().strip().splitlines()[-1]); b=d['batch']; r=b['roundtrip']
print('SB_NIB=$v', 'C2', d['value'], 'batch blocks/s', b['blocks_per_s'], 'C5', r['roundtrip_blocks_per_s'], 'dec ms', r['dec_ms_per_step'], 'bit_exact', r['bit_exact'], 'batch precision', (b.get('precision') or {}).get('margin_factor'))"
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
