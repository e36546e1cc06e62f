#!/bin/bash
# Round 6 call f: VALU issue costs (micro), K1 parity tests, A/B of the current K1 against
# call e's (lib e), counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06f
mkdir -p $OUT
cd $R
timeout -k 10 120 scripts/micro/bin/valu_rates > $OUT/valu_rates.txt 2>&1; echo "valu_rates rc=$?"; cat $OUT/valu_rates.txt
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest ${TESTF:-tests/test_gpu_parity.py} -m gpu -x -v --timeout 200 --timeout-method thread -k "${TESTK:-not nothing}" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
VARIANTS="${VARIANTS:-base e}" ROUNDS=${ROUNDS:-3} CFG=${CFG:-c2} bash scripts/r05_c.sh || exit 1
if [ "${PMC:-1}" = 1 ]; then
  KREGEX=k_tokcount_sl PASSES=2 bash scripts/prof_k1.sh f > /dev/null 2>&1
  python3 scripts/pmc_summary.py gpurun_out/prof_f k_tokcount_sl
fi
