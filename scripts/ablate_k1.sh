#!/bin/bash
# K1 ablation timing (results invalid by design): one bench run per diagnostic build
# lib/libtfidf_hip_abl<N>.so (make -C parallel-systems-mpi-tfidf_amd abl ABL="...").
R=${GRAFT_REPO_ROOT:-/root/repo}
for a in ${ABL:-0}; do
  if [ "$a" = "0" ]; then V=""; else V="abl$a"; fi
  TFIDF_LIB=$V TFIDF_K1_ABLATE=$a timeout -k 10 120 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit > $R/gpurun_out/abl_$a.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/abl_$a.json')); print('ablate', '$a', 'k1 ms', d['roofline']['k1_avg_ms'])"
done
