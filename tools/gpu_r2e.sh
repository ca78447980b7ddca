set -e -o pipefail
O=gpurun_out/r2m
mkdir -p $O
AESFHE_BOOT_MSG_BITS=7 timeout -k 10 100 python3 scratch/evalmod_probe.py > $O/em7.json
for b in 7 8 9; do
  AESFHE_BOOT_MSG_BITS=$b timeout -k 10 100 python3 tools/boot_error_probe.py > $O/p_$b.json
done
timeout -k 10 100 python3 tools/boot_digest.py > $O/digest.json
echo done
