#!/bin/bash
# Round 5: the owner form's aggregation as a radix sort of (bucket, record) pairs: the
# exchange / group GPU tests (TESTK), then configs at 8 shards on the GPU and a kernel trace
# of c4 at 8 shards (rocpd database -> scripts/rocpd_stats.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05g
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
if [ -n "$TESTK" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" $OUT/gpu_tests.log | tail -30; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
for c in ${CFGS:-c4 c5 c3}; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shards8_$c.json')); print('shards8 $c', d['value'], d['ms_per_step'], d.get('exchange_ms_min_over_ranks'), d.get('exchange_mode'))"
done
if [ "${TRACE:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/c4x8 -o run -- python3 bench.py --config c4 --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/c4x8_trace.json 2> $OUT/c4x8_trace.err || { tail -20 $OUT/c4x8_trace.err; exit 1; }
  db=$(find $OUT/c4x8 -name "*.db" | head -1)
  python3 scripts/rocpd_stats.py $db 40 > $OUT/c4x8_kernel_stats.csv && grep -E "k_xb|k_rs|k_owner|k_xcopy|k_keys_by" $OUT/c4x8_kernel_stats.csv
fi
