set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_task.sh r6u bench
echo done
