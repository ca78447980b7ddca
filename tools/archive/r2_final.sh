#!/bin/bash
# Round-2 refresh on the GPU box (through gpurun, from the repo root): the default bench line,
# a rocprofv3 --kernel-trace --stats summary of the C2 bench, the step breakdown of one round.
# Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r2final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/bench_under_rocprof.json 2> $O/trace.err
find $O/trace -name '*kernel_trace.csv' -delete
echo trace done
timeout -k 10 200 python3 tools/step_profile.py > $O/step_profile.json
echo done
