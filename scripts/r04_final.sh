#!/bin/bash
# Round 4 final measurement, part PART (1 or 2) on the committed tree:
#   1: full GPU suite, smoke, the driver's default bench (c2), c3/c4/c5 benches, 8-shard exchange benches
#   2: K1 traffic passes (c2 c4 c5) + c2 kernel trace, the 8-shard exchange benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04final
mkdir -p $OUT
cd $R
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; tail -3 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
  echo "smoke: $(tail -1 $OUT/smoke.log)"
  timeout -k 10 600 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
  tail -1 $OUT/bench_c2.json | cut -c1-400
  for c in c3 c4 c5; do
    timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
    echo "$c: $(tail -1 $OUT/bench_$c.json | cut -c1-160)"
  done
  for c in c5 c3 c4; do
    timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
    echo "shards8 $c: $(tail -1 $OUT/shards8_$c.json | cut -c1-200)"
  done
else
  cd /tmp && export TMPDIR=/tmp
  for c in c2 c4 c5; do
    CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config $c"
    i=0
    for pmc in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/traffic_$c/p$i -o p$i -- $CMD > $OUT/traffic_${c}_p$i.log 2>&1 || { echo "pass $c $pmc failed"; tail -5 $OUT/traffic_${c}_p$i.log; exit 1; }
    done
    echo "traffic $c done"
  done
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c2 -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/kt_c2.log 2>&1 || { echo "trace failed"; exit 1; }
  echo "trace done"
  cd $R
  for c in c5 c3 c4; do
    timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
    echo "shards8 $c: $(tail -1 $OUT/shards8_$c.json | cut -c1-200)"
  done
fi
