#!/bin/bash
# One GPU call (through gpurun, from the repo root): the -m gpu suite, then the default bench
# line.  Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo done
