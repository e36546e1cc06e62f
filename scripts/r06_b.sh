#!/bin/bash
# Round 6 call b: the two-pass K1 (TFIDF_K1=2p) against the oracle (GPU parity suite with the
# mode forced, then the K1-variants test), then an A/B of the default and 2p on c2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06b
mkdir -p $OUT
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  TFIDF_K1=2p timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 120 --timeout-method thread -k "${TESTK:-not k1_variants}" > $OUT/tests_2p.log 2>&1 || { echo "2p TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/tests_2p.log | tail -30; tail -5 $OUT/tests_2p.log; exit 1; }
  echo "2p tests: $(tail -1 $OUT/tests_2p.log)"
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "k1_variants" > $OUT/tests_var.log 2>&1 || { echo "variant TESTS FAILED"; tail -30 $OUT/tests_var.log; exit 1; }
  echo "variants: $(tail -1 $OUT/tests_var.log)"
fi
VARIANTS="${VARIANTS:-base env:TFIDF_K1=2p}" ROUNDS=${ROUNDS:-3} CFG=${CFG:-c2} bash scripts/r05_c.sh
