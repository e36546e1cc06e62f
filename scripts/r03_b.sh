#!/bin/bash
# Round 3: first runs of k_tokcount_lean (quick parity first), A/B bench against the
# round-2 kernel, the GPU test suite, a hip-API trace of a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "golden or variants or edge or boundaries" > $OUT/quick.log 2>&1 || { echo "quick parity failed"; tail -30 $OUT/quick.log; exit 1; }
tail -3 $OUT/quick.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_lean.json 2> $OUT/bench_lean.err \
    || { echo "bench lean failed"; tail -5 $OUT/bench_lean.err; exit 1; }
cat $OUT/bench_lean.json
TFIDF_K1=st timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $OUT/bench_st.json 2> $OUT/bench_st.err \
    || { echo "bench st failed"; tail -5 $OUT/bench_st.err; exit 1; }
cat $OUT/bench_st.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/trace -o tr -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $OUT/trace_bench.json 2> $OUT/trace_bench.err \
    || { echo "trace failed"; tail -5 $OUT/trace_bench.err; exit 1; }
echo done
