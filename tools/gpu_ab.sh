#!/bin/bash
# A/B of the bootstrap between a saved build ($1) and the in-tree build: residue digests,
# pair-bootstrap time, k_lin_mac average (tools/boot_digest.py).  One GPU step per build.
set -e -o pipefail
O=gpurun_out/${2:-ab}
mkdir -p $O
timeout -k 10 200 python3 tools/boot_digest.py $1 > $O/a.json
timeout -k 10 200 python3 tools/boot_digest.py > $O/b.json
cat $O/a.json $O/b.json
