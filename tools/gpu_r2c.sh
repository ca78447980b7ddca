set -e -o pipefail
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fusions.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_sub_ark.log 2>&1
timeout -k 10 300 python3 tools/fusion_bench.py > $O/fusion_bench.json
echo done
