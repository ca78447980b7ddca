# round-6 A/B of InvMixColumns' GF pair renorm (AESFHE_IMC_PAIR_RENORM) on the batch leg's C5 round trip
set -e -o pipefail
O=gpurun_out/${1:-r6im}; mkdir -p $O
for e in ${CFGS:-AESFHE_IMC_PAIR_RENORM=0 AESFHE_NONE=0 AESFHE_IMC_PAIR_RENORM=0 AESFHE_NONE=0}; do
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 2 --detail-json $O/d.json > $O/b.json 2> $O/b.err
  python3 -c "import json; d=json.load(open('$O/d.json')); b=d['batch']; r=b['roundtrip']; print('$e', round(b['blocks_per_s'],1), round(r['enc_ms_per_step'],1), round(r['dec_ms_per_step'],1), round(r['roundtrip_blocks_per_s'],1), r['roundtrip_bit_exact'], (b.get('precision') or {}).get('margin_factor'))"
done
