#!/bin/bash
# Round-3 timeline pass (through gpurun, from the repo root): the C2 round timeline under
# rocprofv3 --kernel-trace (idle gaps by neighbouring kernels, per-family time) and the same
# rounds without the profiler (wall vs host enqueue time per round: is the host the limit?).
# Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r3timeline}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/round_timeline.py run 8 > $O/round_wall.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 tools/round_timeline.py run 8 > $O/round_wall_prof.json
timeout -k 10 120 python3 tools/round_timeline.py analyse $O/round_timeline.json $O/tl > $O/round_timeline_summary.json
echo done
