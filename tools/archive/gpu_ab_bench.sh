#!/bin/bash
# A/B of a saved build ($1) against the in-tree build: bootstrap digests + pair time
# (tools/boot_digest.py) and the C2 bench line (3 steps), each build in its own processes.
set -e -o pipefail
O=gpurun_out/${2:-abb}
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch-states 0 --true-fhe-steps 0"
timeout -k 10 200 python3 tools/boot_digest.py $1 > $O/a_digest.json
timeout -k 10 200 python3 tools/boot_digest.py > $O/b_digest.json
AESFHE_LIB=$1 timeout -k 10 300 python3 $B > $O/a_bench.json
timeout -k 10 300 python3 $B > $O/b_bench.json
AESFHE_LIB=$1 timeout -k 10 300 python3 $B > $O/a2_bench.json
timeout -k 10 300 python3 $B > $O/b2_bench.json
cat $O/a_digest.json $O/b_digest.json
for f in a_bench b_bench a2_bench b2_bench; do python3 -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],3))"; done
