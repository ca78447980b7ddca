set -e -o pipefail
O=gpurun_out/p9; mkdir -p $O
for cfg in "12 4 27" "12 4 23" "12 4 19" "10 4 23" "12 3 27"; do
  set -- $cfg
  AESFHE_BOOT_K=$1 AESFHE_BOOT_R=$2 AESFHE_BOOT_DEG=$3 timeout -k 10 120 python3 tools/evalmod_deg_probe.py >> $O/probe.jsonl
  AESFHE_BOOT_K=$1 AESFHE_BOOT_R=$2 AESFHE_BOOT_DEG=$3 timeout -k 10 120 python3 bench.py --no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --steps 10 | sed "s/^/$1_$2_$3 /" >> $O/bench.txt
done
