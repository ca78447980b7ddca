#!/bin/bash
# Round-3 GPU check (through gpurun, from the repo root): the GPU tests named on the command line
# (default: the whole -m gpu suite), then the default bench line and a rocprofv3 --kernel-trace
# --stats summary of the C2 bench.  Each GPU step has its own limit; the first failure ends it.
set -e -o pipefail
O=gpurun_out/${1:-r3check}
shift || true
TESTS=${*:-tests}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo tests done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/bench_under_rocprof.json 2> $O/trace.err
find $O/trace -name '*kernel_trace.csv' -delete
timeout -k 10 300 python3 tools/launch_census.py > $O/launch_census.json
echo done
