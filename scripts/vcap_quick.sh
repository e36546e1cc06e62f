#!/bin/bash
# K1 stage time vs the initial vocabulary capacity (GPU box): split and fused kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in auto st; do for cap in 131072 262144 1048576; do for load in 50; do
  r=$(TFIDF_K1=$k TFIDF_VCAP=$cap TFIDF_VLOAD=$load timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-emit --no-probe 2>/dev/null) || { echo "fail $k $cap"; exit 1; }
  echo "$k cap=$cap load=$load $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["stage_ms"]["tokcount"], d["k1_work"]["vocab_capacity"], d["value"])')"
done; done; done
