#!/bin/bash
# Round 6 M: the wide DF form (k_df_hist_lds<true>: at most 4 workgroups per resident slot);
# DF tests, c2/c3/c5 benches, a c3 kernel trace, then the full-size property tests (c3: 2.9e9 pairs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06m
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "bin_overflow or wide_form or df_split or vocabulary_boundary" --durations=0 > $OUT/df_tests.log 2>&1 || { echo "DF TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/df_tests.log | tail -20; tail -3 $OUT/df_tests.log; exit 1; }
echo "df tests: $(tail -1 $OUT/df_tests.log)"
for c in c2 c5 c3; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
done
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o kt -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config c3 > $OUT/kt_c3.log 2>&1 ) || { echo "c3 trace failed"; tail -5 $OUT/kt_c3.log; exit 1; }
echo "c3 trace done"
head -12 $OUT/kt_c3/kt_kernel_stats.csv | cut -c1-160
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread -k "full_config_properties" --durations=0 > $OUT/full_tests.log 2>&1 || { echo "FULL TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/full_tests.log | tail -20; tail -3 $OUT/full_tests.log; exit 1; }
echo "full tests: $(tail -1 $OUT/full_tests.log)"
grep -E "s call" $OUT/full_tests.log
