#!/bin/bash
# Live kernel timing (bench.py's in-kernel clock, one launch in 32) against rocprofv3 on the same
# C2 workload: the bench line under rocprofv3 --kernel-trace --stats, the timed window's per-kernel
# averages (tools/trace_window.py), and the bench line alone.  Through gpurun.
set -e -o pipefail
O=gpurun_out/${1:-livecheck}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0"
AESFHE_MARK_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 12 --warmup 1 $B > $O/bench_under_rocprof.json
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
timeout -k 10 120 python3 tools/trace_window.py $O/kernel_stats_timed.json $O/prof
rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 300 python3 bench.py --steps 12 --warmup 1 $B > $O/bench_same_workload.json
echo done
