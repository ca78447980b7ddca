set -e -o pipefail
O=gpurun_out/${1:-r5o}; mkdir -p $O
K=aes-implementation-fhe_amd/libaesfhe_kipf.so
timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_base.json
timeout -k 10 200 python3 tools/enc_digest.py $K > $O/digest_kipf.json
cat $O/digest_*.json
AESFHE_LIB=$K timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_ki.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_kipf.log 2>&1 || { tail -40 $O/pytest_kipf.log; exit 1; }
tail -2 $O/pytest_kipf.log
PASSES=2 bash tools/env_ab.sh ${1:-r5o} AESFHE_LIB=$K -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    c = d['roofline_step']['classes']
    print(cfg[-20:], 'C2', d['value'], 'key_inner', c['key_inner'][:3])
PY
for v in "AESFHE_LIB=$K" "AESFHE_NONE=1"; do
  env $v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 \
      --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --pair-states 64 --pair-stack 64 --pair-steps 1 \
      --detail-json $O/stack_${v##*/}.json > /dev/null
  python3 -c "
import json,sys; d=json.load(open('$O/stack_${v##*/}.json')); bp=d['batch_pairs']
print('$v'[-20:], 'stack ms/pair', round(bp['ms_per_pair'],2), 'key_inner', {k: round(bp['roofline_step']['classes']['key_inner'][k],3) for k in ('frac','avg_us')})"
done
