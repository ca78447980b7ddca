set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_task.sh r6v boot rocwin
echo done
