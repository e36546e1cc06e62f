#!/bin/bash
# bench lines of CFGS (GPU box) then the GPU tests; each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in ${CFGS:-c5 c2}; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe > gpurun_out/b_$cfg.json 2> gpurun_out/b_$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/b_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['stage_ms'])"
done
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
