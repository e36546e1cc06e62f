#!/bin/bash
# K5 timing variants (GPU box): bash scripts/k5_variants.sh [variant ...]
# "main" = lib/libtfidf_hip.so; any other name = lib/libtfidf_hip_<name>.so (make variant).
R=${GRAFT_REPO_ROOT:-/root/repo}
VARS=${@:-main kc64 kc128 kc512}
for cfg in ${CFGS:-c2 c5}; do for v in $VARS; do
  if [ "$v" = "main" ]; then V=""; else V="$v"; fi
  TFIDF_LIB=$V timeout -k 10 120 python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/k5_${cfg}_$v.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/k5_${cfg}_$v.json')); print('$cfg', '$v', d['value'], 'score', d['stage_ms']['score'])"
done; done
