#!/bin/bash
# Round-3 PMC pass (through gpurun, from the repo root).
# 1. FETCH_SIZE / WRITE_SIZE of the dominant kernels over one middle round (tools/r2_pmc_filtered.sh,
#    tools/pmc_round.py), reduced to per-kernel traffic / algorithmic bytes (tools/pmc_reduce.py).
# 2. LAST, once: the full bench command under one FETCH_SIZE pass, to see
#    whether the abort of profiles/r2_pmc_bench_failure.log persists with every launch validated
#    on the host (csrc/launch.h).  Its exit status is recorded, nothing runs after it.
set -e -o pipefail
O=gpurun_out/${1:-r3pmc}
mkdir -p $O
export TMPDIR=/tmp
bash tools/r2_pmc_filtered.sh ${1:-r3pmc}
timeout -k 10 120 python3 tools/pmc_reduce.py "--source=rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (separate runs, --kernel-include-regex on the NTT/conversion/key-switch/lin_mac kernels) over tools/pmc_round.py: one middle encrypt round of the bench workload, one stream, whole process incl. key generation; FETCH_SIZE x2 for 16-B-per-lane reads, x1 for NTT pass 2 dword reads (tools/ntt_pmc_calib.py); L2-miss bytes (MALL hits included), an upper bound on HBM bytes" --alg=$O/pmc_algorithmic.json $O/pmc_traffic_round.json $O/pmc_fetch $O/pmc_write > /dev/null
rm -rf $O/pmc_fetch $O/pmc_write
echo filtered done
rc=0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench -o run -- python3 bench.py --serial --steps 1 --warmup 1 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/pmc_bench.out 2> $O/pmc_bench.err || rc=$?
echo "exit status $rc" > $O/pmc_bench.rc
tail -c 20000 $O/pmc_bench.err > $O/pmc_bench.err.tail || true
find $O/pmc_bench -name '*.csv' -size +1M -delete 2>/dev/null || true
echo "pmc bench rc=$rc"
