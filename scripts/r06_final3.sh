#!/bin/bash
# Round 6 final measurement of the committed tree after the owner-exchange changes (c087d9e):
# full GPU suite, smoke, the driver's default bench (c2) x3, c3/c4/c5 benches, 8-shard
# exchange benches, c2 kernel trace.  K1 and K5 are unchanged since 0fc3d6f (K1 digest
# bba7c88...: its traffic entries stay valid; the c2 counters of r06_final2 stay current).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06final3
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; tail -3 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { echo "bench failed"; tail -20 $OUT/bench_c2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['stage_ms_mean'])"
done
for c in c3 c4 c5; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['traffic'], d['stage_ms_mean'])"
done
for c in c5 c3 c4; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shards8_$c.json')); print('shards8 $c', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_ms_min_over_ranks'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c2 -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config c2 > $OUT/kt_c2.log 2>&1 || { echo "trace c2 failed"; tail -5 $OUT/kt_c2.log; exit 1; }
echo "trace c2 done"
