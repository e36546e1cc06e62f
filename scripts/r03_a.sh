#!/bin/bash
# Round 3, first GPU call: the driver's bench as the FIRST GPU process of a fresh box,
# then a hip-API trace of a short bench (hipMalloc/hipFree between timed steps?), then
# the GPU test suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_fresh.json 2> $OUT/bench_fresh.err \
    || { echo "bench failed"; tail -5 $OUT/bench_fresh.err; exit 1; }
cat $OUT/bench_fresh.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/trace -o tr -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $OUT/trace_bench.json 2> $OUT/trace_bench.err \
    || { echo "trace failed"; tail -5 $OUT/trace_bench.err; exit 1; }
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
