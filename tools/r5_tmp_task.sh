set -e -o pipefail
O=gpurun_out/${1:-r5w}; mkdir -p $O
for pass in 1 2; do for v in 0 1; do
  AESFHE_IMC_GF_LOW=$v timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch-states 1024 --batch-steps 2 \
      --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --detail-json '' > $O/imc_$v.json
  python3 -c "
import json; d=json.loads(open('$O/imc_$v.json').read().strip().splitlines()[-1]); b=d['batch']; r=b['roundtrip']
print('IMC_GF_LOW=$v', 'C2', d['value'], 'batch enc blocks/s', b['blocks_per_s'], 'C5 roundtrip blocks/s', r['roundtrip_blocks_per_s'], 'dec ms', r['dec_ms_per_step'], 'bit_exact', r['bit_exact'])"
done; done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_packed.py tests/test_gpu_reference_paths.py tests/test_gpu_aes.py tests/test_gpu_packed_xor.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dec.log 2>&1 || { tail -40 $O/pytest_dec.log; exit 1; }
tail -2 $O/pytest_dec.log
