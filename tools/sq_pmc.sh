#!/bin/bash
# One rocprofv3 --pmc pass of 8 SQ counters (wave time split into parked / issue-stalled /
# issuing, VALU and LDS instruction counts) over one middle encrypt round of the bench workload
# (tools/pmc_round.py), reduced per kernel family by tools/sq_reduce.py.  Through gpurun.
set -e -o pipefail
O=gpurun_out/${1:-sqpmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    --output-format csv -d $O/sq -o run -- python3 tools/pmc_round.py ${SQ_ARGS:-} > $O/sq.out 2> $O/sq.err
timeout -k 10 120 python3 tools/sq_reduce.py $O/sq_round.json $O/sq > $O/sq_summary.json
echo done
