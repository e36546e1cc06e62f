#!/bin/bash
# K1 time vs vocabulary size (diagnostic): bench --vocab V for each V.
R=${GRAFT_REPO_ROOT:-/root/repo}
for V in ${VS:-1000 50000}; do
  TFIDF_LIB=${LIBV:-} TFIDF_K1_ABLATE=${KABL:-0} timeout -k 10 120 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --vocab $V > $R/gpurun_out/voc_$V.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/voc_$V.json')); print('V', $V, 'lib', '${LIBV:-main}', 'k1 ms', d['roofline']['k1_avg_ms'], 'tokens', d['tokens_per_s'])"
done
