# AESFHE_NTT_SMALL_ROWS (launches below it use 256-thread NTT blocks) A/B on one box: C2 bench
# without the batch / true-FHE legs, two passes over the values.  Run through gpurun.
set -e -o pipefail
O=gpurun_out/p21; mkdir -p $O
for pass in 1 2; do
  for v in 16 0 8 24 32; do
    AESFHE_NTT_SMALL_ROWS=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --steps 10 | sed "s/^/rows=$v /" >> $O/bench.txt
  done
done
