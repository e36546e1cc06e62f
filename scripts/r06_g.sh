#!/bin/bash
# Round 6 call g: the cross-rank long-term check's tests, an A/B of the current K1 against
# call e's (lib e), then SQ counters of the current K1 and of three timing ablations (ablr:
# tokenize only, ablc: no LDS count, ablw: no record writes; wrong output by design).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06g
mkdir -p $OUT
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "${TESTK:-long or cross}" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error|assert|RESULT" $OUT/gpu_tests.log | tail -30; tail -5 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
VARIANTS="${VARIANTS:-base e}" ROUNDS=${ROUNDS:-3} CFG=${CFG:-c2} bash scripts/r05_c.sh || exit 1
for v in ${PV:-base ablr ablc ablw}; do
  L=$v; [ $v = base ] && L=""
  TFIDF_LIB=$L KREGEX=k_tokcount_sl PASSES=2 bash scripts/prof_k1.sh g_$v > /dev/null 2>&1
  echo "## $v"; python3 scripts/pmc_summary.py gpurun_out/prof_g_$v k_tokcount_sl | grep -E "INSTS_VALU|INSTS_SALU|INSTS_LDS|WAVE_CYCLES|WAIT_ANY|BANK"
done
