#!/bin/bash
# Round 6 Z: the tree after the preprocessor clean-up: GPU suite, smoke, default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06z
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; tail -3 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 600 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'])"
