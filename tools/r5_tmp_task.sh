set -e -o pipefail
O=gpurun_out/${1:-r5k}; mkdir -p $O
A=aes-implementation-fhe_amd/libaesfhe_ab0.so
timeout -k 10 200 python3 tools/enc_digest.py $A > $O/digest_old.json
timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_new.json
cat $O/digest_old.json $O/digest_new.json
PASSES=2 bash tools/env_ab.sh ${1:-r5k} AESFHE_LIB=$A -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    c = d['roofline_step']['classes']
    print(cfg[-12:], 'C2', d['value'], 'launches', d['roofline_step']['launches_per_step'],
          'base_convert [frac, avg_us, span]', c['base_convert'][:3])
PY
for k in 0 1; do
  AESFHE_LIN_MAC_NB1=$k timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 \
      --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --pair-states 64 --pair-stack 64 --pair-steps 1 \
      --detail-json $O/stack_nb1_$k.json > $O/stack_nb1_$k.line
done
python3 - $O <<'PY'
import json, sys
for k in (0, 1):
    d = json.load(open(f'{sys.argv[1]}/stack_nb1_{k}.json'))
    bp = d['batch_pairs']
    print('NB1', k, 'C2', d['value'], 'pairs', json.dumps({x: bp.get(x) for x in ('value', 'unit', 'ms_per_pair', 'ms_per_step')}),
          'lin_mac', bp['roofline_step']['classes'].get('lin_mac'), 'key_inner', bp['roofline_step']['classes'].get('key_inner'))
PY
SQ_ARGS="pairs=16" bash tools/sq_pmc.sh ${1:-r5k}/sq16
