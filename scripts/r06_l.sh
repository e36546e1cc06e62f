#!/bin/bash
# Round 6 call l: c4 with k_tokcount_sl over the 32M-slot vocabulary table
# (TFIDF_SL_MAXCAP=2^25) against k_tokcount_vs (the default above 4M slots), with the c4 parity
# tests run on the sl form first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06l
mkdir -p $OUT
cd $R
TFIDF_SL_MAXCAP=33554432 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "c4" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
VARIANTS="${VARIANTS:-base env:TFIDF_SL_MAXCAP=33554432}" ROUNDS=${ROUNDS:-2} CFG=c4 bash scripts/r05_c.sh || exit 1
