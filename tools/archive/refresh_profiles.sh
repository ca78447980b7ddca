#!/bin/bash
# Regenerates the round's profile artifacts on the GPU box (run through gpurun from the repo
# root); outputs under gpurun_out/refresh/, copied into profiles/ by hand.  Every GPU step has
# its own time limit and the steps are chained: the first failure ends the script.
set -e -o pipefail
O=gpurun_out/refresh
mkdir -p $O
export TMPDIR=/tmp
KIDS=key_inner,base_convert,ntt_cols_fwd,ntt_rows_fwd
SRC="rocprofv3 --pmc FETCH_SIZE (x2 for 16-B-per-lane reads, x1 for NTT pass 2 dword reads, tools/ntt_pmc_calib.py) / WRITE_SIZE passes on tools/ks_probe.py, whole process (bench parameter set); the traffic/algorithmic ratio of the same launches is applied to the bench launches (rocprofv3 counter collection segfaults on the full bench)"

# 1. algorithmic bytes of the probe (engine accounting from the first launch on)
AESFHE_PROFILE_FROM_START=$KIDS timeout -k 10 120 python3 tools/ks_probe.py > $O/pmc_probe_algorithmic.json
# 2. HBM traffic of the same probe: one counter per pass
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 tools/ks_probe.py > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 tools/ks_probe.py > /dev/null
timeout -k 10 60 python3 tools/pmc_reduce.py "--source=$SRC" --alg=$O/pmc_probe_algorithmic.json $O/pmc_traffic.json $O/pmc_fetch $O/pmc_write > /dev/null
# 3. kernel trace + stats of the C2 bench (one timed step)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 \
    --no-cpu-baseline --batch-states 0 --traffic-json $O/pmc_traffic.json > $O/bench_under_rocprof.json
timeout -k 10 60 python3 tools/trace_gaps.py $O/trace_gaps.json $O/prof
# 4. the unperturbed bench line (C2 + batch + CPU baseline)
timeout -k 10 400 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench.json
# 5. bootstrap and step breakdowns
timeout -k 10 200 python3 tools/boot_profile.py > $O/boot_profile.json
timeout -k 10 200 python3 tools/boot_kstats.py > $O/boot_kernel_classes.json
timeout -k 10 200 python3 tools/step_profile.py > $O/step_profile.json
timeout -k 10 200 python3 tools/microbench.py > $O/microbench.json
echo done
