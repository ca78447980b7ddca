# round-6 A/B of the C2 set's key-switching digits at fresh level 8 (bench.py --dnum), same box, interleaved
set -e -o pipefail
O=gpurun_out/${1:-r6dn}; mkdir -p $O
for d in ${DNUMS:-4 3 5 4 3 5}; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --steps 10 --detail-json "" --dnum $d > $O/b.json 2> $O/b.err || { echo "dnum $d failed"; tail -2 $O/b.err; continue; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('dnum $d', d['value'], d['precision']['margin_factor'], d['config']['params'])"
done
