#!/bin/bash
# Round 5: (1) K1 timing ablations (A/B of variant libraries, c2), (2) the comm_init deadline
# diagnostic, (3) the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05b
mkdir -p $OUT
cd $R
for r in 1 2; do
  for v in base abl_w abl_c abl_v abl_cv abl_r; do
    L=$v; [ $v = base ] && L=""
    TFIDF_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $OUT/ab.json 2>$OUT/ab.err || { echo "fail $v"; tail -5 $OUT/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/ab.json')); s=d['stage_ms_mean']; print('$v', d['value'], 'k1', s['tokcount'], 'score', s['score'], 'df', s['df'], 'idf', d['idf'])"
  done
done
TFIDF_COMM_TIMEOUT_S=3 timeout -k 5 40 python3 -u scripts/r05_diag_init.py > $OUT/diag_init.log 2>&1
echo "diag_init rc=$?"; grep -E "^ *[0-9]+\.[0-9]+ |tfidf:" $OUT/diag_init.log | tail -8
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" $OUT/gpu_tests.log | tail -30; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
