#!/bin/bash
# K1 ablation timing (results invalid by design): one bench run per TFIDF_K1_ABLATE mask.
R=${GRAFT_REPO_ROOT:-/root/repo}
for a in ${ABL:-0 1 2 3 4}; do
  TFIDF_K1_ABLATE=$a timeout -k 10 120 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/abl_$a.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/abl_$a.json')); print('ablate', $a, 'k1 ms', d['roofline']['k1_avg_ms'])"
done
