# A/B of the multi-input batched EvalMod (AESFHE_EVALMOD_BATCH): full-slot bootstrap digests
# (tools/boot_digest.py), the packed sparse bootstrap digest + time, the bench with its batch
# leg; then the bootstrap / packed GPU tests.  Run through gpurun from the repo root.
set -e -o pipefail
O=gpurun_out/p17; mkdir -p $O
for b in 1 0; do
  AESFHE_EVALMOD_BATCH=$b timeout -k 10 120 python3 tools/boot_digest.py | sed "s/^/batch=$b /" >> $O/digest.txt
  AESFHE_EVALMOD_BATCH=$b timeout -k 10 120 python3 tools/evalmod_deg_probe.py >> $O/probe.jsonl
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_boot_parity.py tests/test_gpu_bootstrap.py tests/test_gpu_packed.py tests/test_gpu_packed_xor.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for b in 1 0; do
  AESFHE_EVALMOD_BATCH=$b timeout -k 10 300 python3 bench.py --no-cpu-baseline --true-fhe-steps 0 | sed "s/^/batch=$b /" >> $O/bench.txt
done
