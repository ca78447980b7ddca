set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_task.sh r6j census boot
O=gpurun_out/r6j
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum --output-format csv -d $O/wr_smoke -o run -- python3 -c "import __graft_entry__ as g; g.smoke()" > $O/wr_smoke.out 2> $O/wr_smoke.err || echo "smoke-under-WRREQ rc=$?" > $O/wr_smoke_rc.txt
wc -l $O/wr_smoke/run_counter_collection.csv > $O/wr_smoke_rows.txt 2>&1 || true
rm -rf $O/wr_smoke
echo done
