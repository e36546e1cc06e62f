#!/bin/bash
# Stage times per diagnostic library variant (lib/libtfidf_hip_<v>.so; "main" = product).
R=${GRAFT_REPO_ROOT:-/root/repo}
for v in ${VARS:-main}; do
  if [ "$v" = "main" ]; then V=""; else V="$v"; fi
  TFIDF_LIB=$V timeout -k 10 120 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit > $R/gpurun_out/sv_$v.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/sv_$v.json')); print('variant', '$v', 'total', d['device_ms_per_step'], d['stage_ms'])"
done
