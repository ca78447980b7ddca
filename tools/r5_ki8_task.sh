set -e -o pipefail
O=gpurun_out/r5d; mkdir -p $O
AESFHE_KI8=0 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_ki16.json
AESFHE_KI8=1 timeout -k 10 200 python3 tools/enc_digest.py > $O/digest_ki8.json
cat $O/digest_ki16.json $O/digest_ki8.json
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_ki.py tests/test_gpu_fused_giant.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_ki.log 2>&1 || { tail -40 $O/pytest_ki.log; exit 1; }
tail -2 $O/pytest_ki.log
PASSES=2 bash tools/env_ab.sh r5d AESFHE_KI8=0 AESFHE_KI8=1
for k in 0 1; do AESFHE_KI8=$k timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch-states 1024 --batch-steps 2 --no-batch-roundtrip --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0 --detail-json $O/batch_ki$k.json > $O/batch_ki$k.line; done
