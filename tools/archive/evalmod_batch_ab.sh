# A/B of the batched EvalMod baby steps (AESFHE_EVALMOD_BATCH): bootstrap digest + time, bench,
# alternating; then the bootstrap parity tests.  Run through gpurun from the repo root.
set -e -o pipefail
O=gpurun_out/p12; mkdir -p $O
for b in 1 0 1 0; do
  AESFHE_EVALMOD_BATCH=$b timeout -k 10 120 python3 tools/evalmod_deg_probe.py >> $O/probe.jsonl
  AESFHE_EVALMOD_BATCH=$b timeout -k 10 120 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --steps 10 | sed "s/^/batch=$b /" >> $O/bench.txt
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boot_parity.py tests/test_gpu_bootstrap.py -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1
