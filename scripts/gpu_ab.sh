#!/bin/bash
# Build on the box, then A/B the K1 kernels on the c2 bench (default = tokcount_st, vs = round 1)
# and run the GPU tests.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 make -j16 -C parallel-systems-mpi-tfidf_amd > gpurun_out/make.log 2>&1 || { echo "make failed"; tail -30 gpurun_out/make.log; exit 1; }
for k1 in ${K1_LIST:-auto vs}; do
  TFIDF_K1=$k1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-probe --no-emit ${BENCH_ARGS:-} > gpurun_out/bench_$k1.json 2> gpurun_out/bench_$k1.err || { echo "bench $k1 failed"; tail -30 gpurun_out/bench_$k1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$k1.json'));print('$k1', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms'])"
done
if [ -n "${PYTEST_SEL:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_SEL} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -25 gpurun_out/gpu_tests.log
  exit $rc
fi
