#!/bin/bash
# Round 6 N: DF histogram loop schedule A/B (c2, c3): default (ranks stored after the next
# iteration's loads, unconditional buffer loads/stores, 12 records in flight) against the
# committed loop (dfhead), the same schedule with 16 in flight (dfb16), and stores at the
# end of the iteration (dfnp); then the DF tests on the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06n
mkdir -p $OUT
cd $R
for rnd in 1 2; do
  for v in default dfhead dfb16 dfnp; do
    L=""; [ $v != default ] && L=$v
    TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 20 --warmup 3 > $OUT/c2_${v}_$rnd.json 2> $OUT/c2_${v}_$rnd.err || { echo "bench $v failed"; tail -5 $OUT/c2_${v}_$rnd.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_${v}_$rnd.json')); s=d['stage_ms_mean']; print('c2 $v', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
  done
done
for v in default dfhead dfb16; do
  L=""; [ $v != default ] && L=$v
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 3 --warmup 1 --config c3 > $OUT/c3_$v.json 2> $OUT/c3_$v.err || { echo "bench c3 $v failed"; tail -5 $OUT/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$v.json')); s=d['stage_ms_mean']; print('c3 $v', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread -k "bin_overflow or wide_form or df_split or vocabulary_boundary or full_config or c3_sharded or golden" > $OUT/df_tests.log 2>&1 || { echo "DF TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/df_tests.log | tail -20; tail -3 $OUT/df_tests.log; exit 1; }
echo "df tests: $(tail -1 $OUT/df_tests.log)"
