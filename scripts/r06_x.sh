#!/bin/bash
# Round 6 X: config 4's K1 chunk size (CHUNK_BYTES, the high-cardinality chunk of
# tokcount_sl / vs): 12 KB (default) against 8, 16 and 24 KB
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06x
mkdir -p $OUT
cd $R
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; w=d.get('k1_work',{}); print('$2 $1', d['value'], d['ms_per_step'], 'k1', s['tokcount'], 'vocab', s['vocab'], 'merge', s['merge'], 'score', s['score'], 'partial', w.get('partial_records'))"
}
for rnd in 1 2; do
  for v in default cb8 cb16 cb24; do run $v c4 10 2 $rnd || exit 1; done
done
