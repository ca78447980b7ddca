set -e -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_gpu_renorm_pool.py tests/test_gpu_packed_xor.py tests/test_gpu_reference_paths.py tests/test_gpu_packed.py tests/test_gpu_aes.py tests/test_gpu_conj_renorm.py" bash tools/gpu_task.sh r6i tests
PASSES=2 bash tools/env_ab.sh r6i "-" "AESFHE_RENORM_POOL=0"
echo done
