#!/bin/bash
# live kernel-average sampling check: the C2 headline leg with the live in-kernel timing on every
# launch (--profile-every 1) and one launch in 32 (default), then the every-launch leg under
# rocprofv3 with the timed region marked (tools/trace_window.py)
set -e -o pipefail
O=gpurun_out/${1:-r3liveavg}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --steps 12 --warmup 1"
timeout -k 10 300 python3 bench.py $B --profile-every 1 > $O/bench_every1.json
timeout -k 10 300 python3 bench.py $B > $O/bench_every32.json
AESFHE_MARK_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $B --profile-every 1 > $O/bench_every1_under_rocprof.json
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
timeout -k 10 120 python3 tools/trace_window.py $O/kernel_stats_timed.json $O/prof
rm -f $O/prof/run_kernel_trace.csv
echo done
