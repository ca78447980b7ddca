# round-6 true-FHE A/B batch (one gpurun call): the true-FHE tests, then tools/fhe_profile.py per setting
set -e -o pipefail
O=gpurun_out/${1:-r6y}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_true_fhe.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_fhe.log 2>&1
tail -2 $O/pytest_fhe.log
run() { tag=$1; shift; env $ENVS timeout -k 10 300 python3 tools/fhe_profile.py "$@" > $O/fhe_$tag.json 2> $O/fhe_$tag.err; echo "$tag $(cat $O/fhe_$tag.json)"; }
ENVS="AESFHE_NONE=0" run quad_12_4 2 12 4
ENVS="AESFHE_FHE_QUAD=0" run noquad_12_4 2 12 4
ENVS="AESFHE_NONE=0" run quad_11_4 2 11 4
