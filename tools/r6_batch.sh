set -e -o pipefail
export TMPDIR=/tmp
PASSES=3 bash tools/env_ab.sh r6r "-" "AESFHE_NTT_FWD8=1"
echo done
