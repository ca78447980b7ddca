#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the bench's dominant kernels over one middle round of the bench
# workload (tools/pmc_round.py; the full bench aborts inside rocprofv3's counter collection,
# profiles/r2_pmc_bench_failure.log), plus the engine's algorithmic bytes of the same launches.
set -e -o pipefail
O=gpurun_out/${1:-pmcf}
mkdir -p $O
export TMPDIR=/tmp
KIDS=key_inner,base_convert,ntt_cols_fwd,ntt_rows_fwd,ntt_rows_inv,ntt_cols_inv,lin_mac
RX='k_ntt1_fwd|k_ntt2_fwd|k_ntt1_inv|k_ntt2_inv|k_lin_mac|k_base_convert|k_key_inner'
B="${B:-tools/pmc_round.py}"
AESFHE_PROFILE_FROM_START=$KIDS timeout -k 10 200 python3 $B $O/pmc_algorithmic.json > $O/pmc_alg.out
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_fetch -o run -- python3 $B > $O/pmc_fetch.out 2> $O/pmc_fetch.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_write -o run -- python3 $B > $O/pmc_write.out 2> $O/pmc_write.err
echo done
