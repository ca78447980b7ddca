#!/bin/bash
# live kernel averages by dispatch-stamped HIP event pairs (AESFHE_PROF_EVENTS=1) against the
# rocprofv3 timed window of the same launches, and without the profiler
set -e -o pipefail
O=gpurun_out/${1:-r3evtavg}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --steps 12 --warmup 1"
AESFHE_PROF_EVENTS=1 timeout -k 10 300 python3 bench.py $B > $O/bench_events.json
AESFHE_PROF_EVENTS=1 AESFHE_MARK_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $B > $O/bench_events_under_rocprof.json
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
timeout -k 10 120 python3 tools/trace_window.py $O/kernel_stats_timed.json $O/prof
rm -f $O/prof/run_kernel_trace.csv
echo done
