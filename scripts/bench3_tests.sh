cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2 3; do
  out=$(timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-emit --no-probe 2>/dev/null) || { echo fail; exit 1; }
  echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['device_ms_per_step'], d['stage_ms']['tokcount'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; exit $rc
