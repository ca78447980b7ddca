set -e -o pipefail
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_reference_paths.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_refpaths.log 2>&1
timeout -k 10 900 python3 tools/cpu_round.py --full > $O/cpu_round.json 2> $O/cpu_round.err
echo done
