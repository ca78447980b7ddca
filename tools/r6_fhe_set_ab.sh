# round-6 true-FHE set A/B at the renorm floor 1: tools/fhe_profile.py per fresh level (dnum 4)
set -e -o pipefail
O=gpurun_out/${1:-r6fs}; mkdir -p $O
for L in ${LEVELS:-12 11 12 11}; do
  timeout -k 10 300 python3 tools/fhe_profile.py 2 $L 4 > $O/fhe_$L.json 2> $O/fhe_$L.err || { echo "L $L failed"; tail -2 $O/fhe_$L.err; continue; }
  python3 -c "import json; d=json.load(open('$O/fhe_$L.json')); print('L $L', d['ms_per_encrypt'], d['rounds_per_s'], d['verified'], d['precision'])"
done
