# round-6 A/B of the renorm floor (AESFHE_RENORM_FLOOR) with the C2 set's fresh level one lower
set -e -o pipefail
O=gpurun_out/${1:-r6fl}; mkdir -p $O
ARGS="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 10 --detail-json ''"
for cfg in ${CFGS:-"AESFHE_NONE=0:9" "AESFHE_RENORM_FLOOR=1:8"}; do
  e=${cfg%%:*}; L=${cfg##*:}
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 10 --detail-json "" --fresh-level $L > $O/b.json 2> $O/b.err || { echo "$cfg failed"; tail -3 $O/b.err; continue; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['launches_per_encrypt'], d['precision']['margin_factor'], d['config']['params']['log2_pq'])"
done
