set -e -o pipefail
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 200 python3 tools/boot_low_stages.py 32 $O/std.json > $O/std.txt 2>&1
AESFHE_DEBUG_BOOT_FLOOR=7 timeout -k 10 200 python3 tools/boot_low_stages.py 32 $O/low.json > $O/low.txt 2>&1
cat $O/std.txt $O/low.txt
python3 - <<'PY'
import json
import numpy as np
a = json.load(open('gpurun_out/r5h/std.json')); b = json.load(open('gpurun_out/r5h/low.json'))
for k in a:
    x = np.array(a[k]['re']) + 1j * np.array(a[k]['im']); y = np.array(b[k]['re']) + 1j * np.array(b[k]['im'])
    print('stage', k, 'levels', a[k]['level'], b[k]['level'], 'max|std|', round(float(np.abs(x).max()), 4), 'max|low|', round(float(np.abs(y).max()), 4),
          'max|std-low|', float(np.abs(x - y).max()), 'ratio', (y[:4] / x[:4]).round(4).tolist())
PY
