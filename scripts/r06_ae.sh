#!/bin/bash
# sender-side bucketing of the owner exchange: multi-rank tests, then at 8 shards on one GPU
# xold (before c087d9e), sort (TFIDF_XSSB=0: c087d9e's owner-side bucket sort), default (ssb)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ae
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > $OUT/mr_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/mr_tests.log | tail -20; tail -3 $OUT/mr_tests.log; exit 1; }
echo "multirank tests: $(tail -1 $OUT/mr_tests.log)"
run() {   # variant config tag
  local L="" X=""; [ $1 = xold ] && L=xold; [ $1 = sort ] && X=0
  TFIDF_LIB=$L TFIDF_XSSB=$X timeout -k 10 300 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $2 > $OUT/$2_$1_$3.json 2> $OUT/$2_$1_$3.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$3.json')); print('$2 $1', d['value'], d['ms_per_step'], 'xchg', d['exchange_ms'], 'min', d['exchange_ms_min_over_ranks'])"
}
for rnd in 1 2 3; do
  for v in xold sort default; do run $v c4 $rnd || exit 1; done
done
for c in c5 c3; do
  for v in xold sort default; do run $v $c 1 || exit 1; done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config c4 > $OUT/kt.json 2> $OUT/kt.err || { echo "trace failed"; tail -5 $OUT/kt.err; exit 1; }
F=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/xchg_timeline.py $F > $OUT/xchg_timeline.txt && tail -22 $OUT/xchg_timeline.txt
