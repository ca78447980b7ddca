#!/bin/bash
# Round-3 profiling pass (through gpurun, from the repo root): the launch census per engine op of
# one middle round, the GPU timeline of 8 rounds (rocprofv3 kernel trace -> concurrency of the
# branch streams, idle gaps), then the parity tests the oracle changes touch.  Each GPU step has
# its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r3prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/launch_census.py --by-op > $O/census_by_op.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 tools/round_timeline.py run 8 > $O/timeline_run.json
timeout -k 10 120 python3 tools/round_timeline.py analyse $O/timeline.json $O/tl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boot_parity.py tests/test_gpu_lut.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1
echo done
