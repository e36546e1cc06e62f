#!/bin/bash
# Round 6 V: LSD radix sort tile of 4096 keys (rs16: RS_IT 16) against 2048 (default); c4
# (vocabulary + 6.8 M partial records), c5, c3, c2
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06v
mkdir -p $OUT
cd $R
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'vocab', s['vocab'], 'merge', s['merge'], 'df', s['df'], 'order', s['order'])"
}
for rnd in 1 2; do
  for v in default rs16; do run $v c4 10 2 $rnd || exit 1; done
done
for c in c5 c2; do
  for v in default rs16; do run $v $c 10 2 1 || exit 1; done
done
for v in default rs16; do run $v c3 3 1 1 || exit 1; done
