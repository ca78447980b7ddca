set -e -o pipefail
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 300 python3 scratch/fhe_err_probe3.py 256 > $O/err3.txt 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_true_fhe.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_fhe.log 2>&1
timeout -k 10 400 python3 tools/true_fhe_bench.py > $O/true_fhe_bench.json
echo done
