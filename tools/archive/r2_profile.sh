#!/bin/bash
# Round-2 profiling pass on the GPU box (through gpurun, from the repo root):
#  1. kernel trace + stats of the C2 bench (rocprofv3 --kernel-trace --stats);
#  2. step / bootstrap breakdowns;
#  3. HBM traffic of the BENCH itself: one FETCH_SIZE pass and one WRITE_SIZE pass (separate
#     runs, --serial: one stream) over `bench.py --steps 1 --warmup 1 --batch-states 0`, and
#     the engine's algorithmic bytes of exactly the same launches (the same command without
#     the profiler, AESFHE_PROFILE_FROM_START + --whole-stats), reduced by tools/pmc_reduce.py.
# Each GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r2prof}
mkdir -p $O
export TMPDIR=/tmp
KIDS=key_inner,base_convert,ntt_cols_fwd,ntt_rows_fwd,ntt_rows_inv,ntt_cols_inv,lin_mac
B="bench.py --serial --steps 1 --warmup 1 --no-cpu-baseline --batch-states 0"
SRC="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (separate runs) over python3 $B (whole process, one stream); FETCH_SIZE x2 for 16-B-per-lane reads, x1 for NTT pass 2 dword reads (tools/ntt_pmc_calib.py); FETCH_SIZE counts Infinity-Cache (MALL) hits as well, so these are L2-miss bytes, an upper bound on HBM bytes; algorithmic bytes of the same launches from the engine (AESFHE_PROFILE_FROM_START, --whole-stats)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --batch-states 0 > $O/bench_under_rocprof.json 2> $O/trace.err
find $O/trace -name '*kernel_trace.csv' -delete
timeout -k 10 200 python3 tools/step_profile.py > $O/step_profile.json
timeout -k 10 200 python3 tools/boot_kstats.py --pair > $O/boot_pair_kernel_classes.json
AESFHE_PROFILE_FROM_START=$KIDS timeout -k 10 200 python3 $B --whole-stats $O/pmc_bench_algorithmic.json > $O/pmc_alg_bench.json
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $B > $O/pmc_fetch.out 2> $O/pmc_fetch.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $B > $O/pmc_write.out 2> $O/pmc_write.err
timeout -k 10 100 python3 tools/pmc_reduce.py "--source=$SRC" --alg=$O/pmc_bench_algorithmic.json $O/pmc_traffic_bench.json $O/pmc_fetch $O/pmc_write > /dev/null
echo done
