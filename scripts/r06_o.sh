#!/bin/bash
# Round 6 O: DF loop with 32-bit relative indices and buffer gathers (default, 105 VGPRs,
# no spills) against r06n's best (dfb16: 128 VGPRs, 5 spilled) and the committed loop (dfhead)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06o
mkdir -p $OUT
cd $R
for rnd in 1 2; do
  for v in default dfb16 dfhead; do
    L=""; [ $v != default ] && L=$v
    TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 3 --warmup 1 --config c3 > $OUT/c3_${v}_$rnd.json 2> $OUT/c3_${v}_$rnd.err || { echo "bench c3 $v failed"; tail -5 $OUT/c3_${v}_$rnd.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_${v}_$rnd.json')); s=d['stage_ms_mean']; print('c3 $v', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
    TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 20 --warmup 3 > $OUT/c2_${v}_$rnd.json 2> $OUT/c2_${v}_$rnd.err || { echo "bench $v failed"; tail -5 $OUT/c2_${v}_$rnd.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_${v}_$rnd.json')); s=d['stage_ms_mean']; print('c2 $v', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread -k "bin_overflow or wide_form or df_split or vocabulary_boundary or full_config or c3_sharded or golden or variants" > $OUT/df_tests.log 2>&1 || { echo "DF TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/df_tests.log | tail -20; tail -3 $OUT/df_tests.log; exit 1; }
echo "df tests: $(tail -1 $OUT/df_tests.log)"
