set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in auto split; do
  TFIDF_K1=$k timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-emit --no-probe > gpurun_out/c4_$k.json 2> gpurun_out/c4_$k.err || { echo "c4 $k failed"; tail -5 gpurun_out/c4_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_$k.json')); print('$k', d['value'], d['stage_ms'], d['k1_work'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
