#!/bin/bash
# owner exchange A/B at 8 shards on one GPU: xold (HEAD before: k_keys_by_rank, per-word
# k_xcopy search), default (keys from the vocabulary sort, tiled k_xcopy, LDS segment search),
# xb256 (default + owner buckets of <= 256 records on average: 20 KB of LDS, 8 per CU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ad
mkdir -p $OUT
cd $R
TFIDF_LIB=xb256 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/mr_xb256.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/mr_xb256.log | tail -20; tail -3 $OUT/mr_xb256.log; exit 1; }
echo "multirank xb256: $(tail -1 $OUT/mr_xb256.log)"
run() {   # variant config tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $2 > $OUT/$2_$1_$3.json 2> $OUT/$2_$1_$3.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$3.json')); print('$2 $1', d['value'], d['ms_per_step'], 'xchg', d['exchange_ms'], 'min', d['exchange_ms_min_over_ranks'])"
}
for rnd in 1 2 3; do
  for v in xold default xb256; do run $v c4 $rnd || exit 1; done
done
for c in c5 c3; do
  for v in xold default xb256; do run $v $c 1 || exit 1; done
done
