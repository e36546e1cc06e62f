#!/bin/bash
# Round 6 call h: the whole GPU suite on the current tree, then a c2 bench and smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06h
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "BENCH FAILED"; tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c2.json')); print(d['value'], d['ms_per_step'], d['roofline'], d.get('stage_ms_mean'))"
