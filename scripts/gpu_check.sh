#!/bin/bash
# One GPU-box pass: rebuild from source (build/ is not uploaded), a short bench, the GPU tests.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 make -j16 -C parallel-systems-mpi-tfidf_amd > gpurun_out/make.log 2>&1 || { echo "make failed"; tail -30 gpurun_out/make.log; exit 1; }
echo "build ok"
timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
