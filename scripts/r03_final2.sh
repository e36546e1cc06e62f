#!/bin/bash
# Round 3 final evidence after the DF balance change: all GPU tests, the driver's default
# bench and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03final2}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-probe > $OUT/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_c2.log; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_c2.csv
echo done
