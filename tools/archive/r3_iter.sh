#!/bin/bash
# Round-3 iteration pass (through gpurun, from the repo root): the GPU tests that the change under
# test touches, the launch census (per step and per engine op), the default bench line, and (AB=1)
# the headline leg again with the live kernel-timing sample off.  Each GPU step has its own limit;
# the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r3iter}
shift || true
TESTS=${*:-tests}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo tests done
timeout -k 10 300 python3 tools/launch_census.py > $O/launch_census.json
timeout -k 10 300 python3 tools/launch_census.py --by-op > $O/census_by_op.json
echo census done
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
if [ "${AB:-0}" = 1 ]; then
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/bench_sampled.json 2> $O/bench_sampled.err
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --profile-every 1000000000 > $O/bench_nosample.json 2> $O/bench_nosample.err
fi
echo done
