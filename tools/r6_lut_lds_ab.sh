# round-6 A/B of the LDS-staged bivariate LUT kernel (AESFHE_LUT_LDS): residue digests of a C2 encrypt either way
# (bit identity), the LUT / stacked tests, then the C2 leg interleaved
set -e -o pipefail
O=gpurun_out/${1:-r6ll}; mkdir -p $O
AESFHE_LUT_LDS=0 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_off.txt
timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_on.txt
cmp $O/digest_off.txt $O/digest_on.txt && echo "digests identical"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lut.py tests/test_gpu_stacked.py tests/test_gpu_packed_xor.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
PASSES=2 bash tools/env_ab.sh ${1:-r6ll} "AESFHE_LUT_LDS=0" "-"
python3 -c "
import json
for l in open('$O/bench.txt'):
    cfg, js = l.split(' ',1); d=json.loads(js); print(cfg, d['value'], d['launches_per_encrypt'])"
