set -e -o pipefail
O=gpurun_out/${1:-r5ff}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aes.py tests/test_gpu_packed_xor.py tests/test_gpu_reference_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_quick.log 2>&1 || { tail -40 $O/pytest_quick.log; exit 1; }
tail -1 $O/pytest_quick.log
PASSES=2 bash tools/env_ab.sh ${1:-r5ff} AESFHE_TTABLE=0 -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    print(cfg, 'C2', d['value'], 'launches', d['launches_per_encrypt'], 'precision', d['precision']['margin_factor'], d['precision']['worst_stage'])
PY
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
