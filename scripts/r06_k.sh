#!/bin/bash
# Round 6 call k: K1 with the simplified CAS outcome test: parity tests, then an A/B against
# the committed K1 (lib c812).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06k
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
VARIANTS="${VARIANTS:-base c812}" ROUNDS=${ROUNDS:-4} CFG=c2 bash scripts/r05_c.sh || exit 1
