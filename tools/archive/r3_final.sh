#!/bin/bash
# Round-3 profile refresh (through gpurun, from the repo root); outputs under gpurun_out/${1:-r3final}/,
# copied into profiles/ as r3_*.  Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r3final}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0"
# 1. the whole GPU suite
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo tests done
# 2. kernel trace + stats of the C2 headline leg, and its bench line (live kernel averages)
AESFHE_MARK_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 12 --warmup 1 $B > $O/bench_under_rocprof.json
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
timeout -k 10 120 python3 tools/trace_window.py $O/kernel_stats_timed.json $O/prof
rm -f $O/prof/run_kernel_trace.csv
# 3. the same workload without the profiler
timeout -k 10 300 python3 bench.py --steps 12 --warmup 1 $B > $O/bench_same_workload.json
echo rocprof done
# 4. the default bench line (C2 + batch + multi-pair + true-FHE + CPU baseline)
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
# 5. breakdowns
timeout -k 10 300 python3 tools/launch_census.py > $O/launch_census.json
timeout -k 10 300 python3 tools/step_profile.py > $O/step_profile.json
timeout -k 10 200 python3 tools/boot_kstats.py --sparse 32 > $O/boot_kstats_sparse32.json
echo done
