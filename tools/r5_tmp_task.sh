set -e -o pipefail
O=gpurun_out/${1:-r5n}; mkdir -p $O
export TMPDIR=/tmp
C2="--no-cpu-baseline --batch-states 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
for v in 0 1; do
  AESFHE_LUT_REG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- \
      python3 bench.py --steps 4 --warmup 1 $C2 > $O/bench_lut$v.json 2> $O/rocprof$v.err
  cp $O/prof$v/run_kernel_stats.csv $O/kernel_stats_lut$v.csv
  rm -rf $O/prof$v
done
python3 - $O <<'PY'
import csv, sys
for v in (0, 1):
    rows = list(csv.DictReader(open(f'{sys.argv[1]}/kernel_stats_lut{v}.csv')))
    for r in rows:
        n = r['Name']
        if 'lut' in n or 'base_convert' in n or 'ntt1_inv' in n:
            print(v, n.split('(')[0][-60:], r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 2), 'total_ms', round(float(r['TotalDurationNs']) / 1e6, 1))
PY
