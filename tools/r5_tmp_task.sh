set -e -o pipefail
O=gpurun_out/${1:-r5u}; mkdir -p $O
PASSES=2 bash tools/env_ab.sh ${1:-r5u} AESFHE_MC_GF_LOW=0 -
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    print(cfg, 'C2', d['value'], 'launches', d['launches_per_encrypt'], 'precision', d['precision']['margin_factor'], d['precision']['worst_stage'])
PY
timeout -k 10 300 python3 tools/mix_profile.py 5 > $O/mix_profile_default_path.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
