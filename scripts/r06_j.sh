#!/bin/bash
# Round 6 call j: the split flow (K5's order beside the DF pass, scores after it): the GPU
# suite, then an A/B against TFIDF_K5_SPLIT=0 on c2 and c5, and a kernel trace of c2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06j
mkdir -p $OUT
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${TESTK:-not nothing}" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
VARIANTS="${VARIANTS:-base env:TFIDF_K5_SPLIT=0}" ROUNDS=${ROUNDS:-3} CFG=c2 bash scripts/r05_c.sh || exit 1
VARIANTS="${VARIANTS:-base env:TFIDF_K5_SPLIT=0}" ROUNDS=1 CFG=c5 bash scripts/r05_c.sh || exit 1
bash scripts/kstats.sh j_c2 --config c2 --no-emit --no-probe
