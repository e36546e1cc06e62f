#!/bin/bash
# Round 6 call e: K1 with fewer VALU per token (fast token-list loop, packed-counter flush):
# the GPU suite, an A/B against round 5's K1 (lib r5) on c2, then K1's SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06e
mkdir -p $OUT
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${TESTK:-not nothing}" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
VARIANTS="${VARIANTS:-base r5}" ROUNDS=${ROUNDS:-3} CFG=${CFG:-c2} bash scripts/r05_c.sh || exit 1
if [ "${PMC:-1}" = 1 ]; then
  KREGEX=k_tokcount_sl PASSES=2 bash scripts/prof_k1.sh e > /dev/null 2>&1
  python3 scripts/pmc_summary.py gpurun_out/prof_e k_tokcount_sl
fi
