#!/bin/bash
# NTT row-pass (pass 2) block size A/B: AESFHE_NTT_P2_NT (forward) / AESFHE_NTT_P2I_NT (inverse) in
# {512, 256, 128} threads (NT / 16 rows per block; pass 1 keeps 512) and AESFHE_NTT_FIN_OCC (the
# finish mode capped at 128 VGPRs).  Per-launch NTT / INTT times vs rows, then the C2 bench leg per
# setting, two passes.  Run through gpurun; each GPU step has its own limit.
set -e -o pipefail
O=gpurun_out/${1:-p2ab}; mkdir -p $O
[ "${SWEEP:-1}" = 1 ] && for v in "512 512" "256 256" "128 128"; do
  set -- $v
  AESFHE_NTT_P2_NT=$1 AESFHE_NTT_P2I_NT=$2 timeout -k 10 120 python3 tools/ntt_rows_sweep.py | sed "s/^/p2nt=$1 p2int=$2 /" >> $O/sweep.txt
done
[ "${SWEEP:-1}" = 1 ] && echo sweep done
for pass in 1 2; do
  for cfg in ${CFGS:-512_512_0 256_512_1 256_512_0 128_512_1 256_256_1 256_128_1}; do
    set -- ${cfg//_/ }
    AESFHE_NTT_P2_NT=$1 AESFHE_NTT_P2I_NT=$2 AESFHE_NTT_FIN_OCC=$3 timeout -k 10 150 python3 bench.py --no-cpu-baseline --batch-states 0 \
        --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --steps 10 | sed "s/^/p2nt=$1 p2int=$2 finocc=$3 /" >> $O/bench.txt
  done
done
echo done
