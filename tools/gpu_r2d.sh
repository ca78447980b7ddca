set -e -o pipefail
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 200 python3 tools/boot_digest.py > $O/digest.json
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bootstrap.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_boot.log 2>&1
echo done
