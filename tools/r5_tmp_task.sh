set -e -o pipefail
O=gpurun_out/${1:-r5aa}; mkdir -p $O
PASSES=3 bash tools/env_ab.sh ${1:-r5aa} - AESFHE_BOOT_DEG=23 AESFHE_BOOT_DEG=21
python3 - "$O/bench.txt" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    cfg, js = ln.split(' ', 1)
    d = json.loads(js)
    print(cfg, 'C2', d['value'], 'launches', d['launches_per_encrypt'], 'precision', d['precision']['margin_factor'], d['precision']['max_err_rad'])
PY
AESFHE_BOOT_DEG=21 timeout -k 10 300 python3 tools/boot_error_probe.py > $O/boot_err_21.json 2> $O/boot_err_21.err
python3 -c "
import json; d=json.load(open('$O/boot_err_21.json')); print('deg 21', {k: round(v['max_err'],6) for k,v in d.items() if isinstance(v, dict) and 'max_err' in v})"
