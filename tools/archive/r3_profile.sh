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
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boot_parity.py tests/test_gpu_sparse_boot.py tests/test_gpu_bootstrap.py tests/test_gpu_batched.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1

timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/bench_fact.json 2> $O/bench_fact.err
AESFHE_NTT_INV_FACT=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 > $O/bench_nofact.json 2> $O/bench_nofact.err
echo ab done
timeout -k 10 200 python3 tools/boot_kstats.py --sparse 32 > $O/boot_kstats_sparse32.json
echo kstats done
