set -e -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_packed_xor.py tests/test_gpu_reference_paths.py tests/test_gpu_packed.py tests/test_gpu_aes.py tests/test_gpu_true_fhe.py" bash tools/gpu_task.sh r6h tests
PASSES=2 bash tools/env_ab.sh r6h "-" "AESFHE_PT_SUM=0" "AESFHE_MC_HOIST=0"
O=gpurun_out/r6h
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum --output-format csv -d $O/wr_tiny -o run -- python3 -c "import torch; x=torch.ones(1<<20, device='cuda'); y=x*2; torch.cuda.synchronize(); print(float(y.sum()))" > $O/wr_tiny.out 2> $O/wr_tiny.err || echo "tiny rc=$?" > $O/wr_tiny_rc.txt
echo done
