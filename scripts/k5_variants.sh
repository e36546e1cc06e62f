R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in c2 c5; do for v in main kc64 kc128 kc512; do
  if [ "$v" = "main" ]; then V=""; else V="$v"; fi
  TFIDF_LIB=$V timeout -k 10 120 python3 $R/bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/k5_${cfg}_$v.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/k5_${cfg}_$v.json')); print('$cfg', '$v', d['value'], 'score', d['stage_ms']['score'])"
done; done
