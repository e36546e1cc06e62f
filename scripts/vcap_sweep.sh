R=${GRAFT_REPO_ROOT:-/root/repo}
for cap in 262144 524288 1048576 2097152; do
  TFIDF_VCAP=$cap TFIDF_VLOAD=30 timeout -k 10 120 python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-emit > $R/gpurun_out/vs_$cap.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/vs_$cap.json')); print('vcap', $cap, 'k1 ms', d['roofline']['k1_avg_ms'], 'total', d['device_ms_per_step'], d['k1_work']['vocab_capacity'])"
done
