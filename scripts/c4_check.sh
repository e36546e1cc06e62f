#!/bin/bash
# c4 bench line (GPU box) then the GPU tests; each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-emit --no-probe > gpurun_out/c4.json 2> gpurun_out/c4.err || { echo "c4 failed"; tail -5 gpurun_out/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c4.json')); print('c4', d['value'], d['ms_per_step'], d['stage_ms'])"
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-emit --no-probe > gpurun_out/c2.json 2> gpurun_out/c2.err || { echo "c2 failed"; tail -5 gpurun_out/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c2.json')); print('c2', d['value'], d['ms_per_step'], d['stage_ms'])"
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
