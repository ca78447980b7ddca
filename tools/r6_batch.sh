set -e -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_renorm_pool.py tests/test_gpu_packed_xor.py tests/test_gpu_reference_paths.py tests/test_gpu_packed.py tests/test_gpu_conj_renorm.py tests/test_gpu_c3.py" bash tools/gpu_task.sh r6k tests
PASSES=2 bash tools/env_ab.sh r6k "-" "AESFHE_SPARSE_DEC=0"
bash tools/gpu_task.sh r6k census boot
O=gpurun_out/r6k
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum --output-format csv -d $O/wr_smoke -o run -- python3 -c "import __graft_entry__ as g; g.smoke()" > $O/wr_smoke.out 2> $O/wr_smoke.err || echo "smoke-under-WRREQ rc=$?" > $O/wr_smoke_rc.txt
wc -l $O/wr_smoke/run_counter_collection.csv > $O/wr_smoke_rows.txt 2>&1 || true
rm -rf $O/wr_smoke
echo done
