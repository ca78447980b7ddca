set -e -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_renorm_pool.py tests/test_gpu_packed_xor.py tests/test_gpu_reference_paths.py" bash tools/gpu_task.sh r6p tests
PASSES=2 bash tools/env_ab.sh r6p "-" "AESFHE_SPARSE_DEC=0"
echo done
