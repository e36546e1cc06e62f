#!/bin/bash
# Round 4, call A: the pruned tree (experimental K1 kernels removed, deadlock-free vocabulary
# insert, per-rank RCCL clique locks, ABI 2): GPU tests, smoke, then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04a
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
cat $OUT/bench.json
