# round-6 stacked-bootstrap packing batch (one gpurun call): the stacked / chunk / C3 tests, then the
# C3 leg (bench.py batch_pairs: 1,024 one-state pairs, 16 stacks of 64) per AESFHE_STACK_PACK
set -e -o pipefail
O=gpurun_out/${1:-r6p}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stacked.py tests/test_gpu_boot_chunk.py tests/test_gpu_c3.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_pack.log 2>&1
tail -2 $O/pytest_pack.log
LEG="--steps 1 --warmup 1 --no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
for g in ${PACKS:-1 4 8}; do
  AESFHE_STACK_PACK=$g timeout -k 10 400 python3 bench.py $LEG > $O/c3_pack$g.json 2> $O/c3_pack$g.err
  python3 -c "import json,sys; d=json.loads(open('$O/c3_pack$g.json').read().strip().splitlines()[-1]); bp=d.get('batch_pairs') or {}; print('pack $g', {k: bp.get(k) for k in ('ms_per_pair','blocks_per_s','vs_c2','verified_against_plaintext_model','pairs')}, 'C2', d['value'])"
done
