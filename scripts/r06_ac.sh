#!/bin/bash
# owner exchange: keys from the vocabulary sort (no k_keys_by_rank), tiled k_xcopy, LDS
# segment search in k_owner_back.  Multi-rank tests, then the c4 8-shard trace and benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ac
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > $OUT/mr_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/mr_tests.log | tail -20; tail -3 $OUT/mr_tests.log; exit 1; }
echo "multirank tests: $(tail -1 $OUT/mr_tests.log)"
for c in c4 c4 c5; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shards8_$c.json')); print('$c', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_ms_min_over_ranks'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config c4 > $OUT/kt.json 2> $OUT/kt.err || { echo "trace failed"; tail -5 $OUT/kt.err; exit 1; }
F=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/xchg_timeline.py $F > $OUT/xchg_timeline.txt && tail -20 $OUT/xchg_timeline.txt
