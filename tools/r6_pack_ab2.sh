set -e -o pipefail
O=gpurun_out/r6p3; mkdir -p $O
LEG="--steps 1 --warmup 1 --no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
for g in 16 32; do
  AESFHE_STACK_PACK=$g timeout -k 10 300 python3 bench.py $LEG --detail-json $O/d$g.json > $O/c3_pack$g.json 2> $O/c3_pack$g.err
  python3 -c "import json; d=json.loads(open('$O/c3_pack$g.json').read().strip().splitlines()[-1]); bp=d['batch_pairs']; print('pack $g', bp['ms_per_pair'], bp['blocks_per_s'], bp['verified_against_plaintext_model'])"
done
