#!/bin/bash
# Round-2 profiling pass on the GPU box (through gpurun, from the repo root): kernel trace +
# stats of the C2 bench, step / bootstrap breakdowns, then FETCH_SIZE / WRITE_SIZE counter
# passes over the bench itself (--serial: one stream).  Each GPU step has its own limit; the
# first failure ends the script.
set -e -o pipefail
O=gpurun_out/${1:-r2prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --batch-states 0 > $O/bench_under_rocprof.json 2> $O/trace.err
timeout -k 10 200 python3 tools/step_profile.py > $O/step_profile.json
timeout -k 10 200 python3 tools/boot_profile.py > $O/boot_profile.json
timeout -k 10 200 python3 tools/boot_kstats.py > $O/boot_kernel_classes.json
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --serial --steps 1 --warmup 1 \
    --no-cpu-baseline --batch-states 0 > $O/pmc_fetch.out 2> $O/pmc_fetch.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --serial --steps 1 --warmup 1 \
    --no-cpu-baseline --batch-states 0 > $O/pmc_write.out 2> $O/pmc_write.err
echo done
