#!/bin/bash
# Quick GPU pass (box): default bench line, kernel-trace stats, then the GPU tests; every
# GPU step under its own time limit, stopping at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-emit ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash scripts/kstats.sh quick --no-emit --no-probe ${BENCH_ARGS:-} || { echo "kstats failed"; exit 1; }
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
