set -e -o pipefail
O=gpurun_out/${1:-r5ee}; mkdir -p $O
PASSES=3 bash tools/env_ab.sh ${1:-r5ee} AESFHE_SHARE_R1=0 -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    print(cfg, 'C2', d['value'], 'launches', d['launches_per_encrypt'], 'precision', d['precision']['margin_factor'])
PY
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_packed_xor.py tests/test_gpu_packed.py tests/test_gpu_aes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
