#!/bin/bash
# Round 6 R: the DF histogram's workgroup count (TFIDF_DF_WGS: 256 = one per CU, 512, default
# = up to four per CU slot) with the pipelined loop; c2 x2, c3
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06r
mkdir -p $OUT
cd $R
run() {   # wgs config steps warmup tag
  local E=""; [ $1 != default ] && E=$1
  TFIDF_DF_WGS=$E timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 wgs=$1', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
}
for rnd in 1 2; do
  for v in default 256 512; do run $v c2 20 3 $rnd || exit 1; done
done
for v in default 256 512; do run $v c3 3 1 1 || exit 1; done
for v in default 256; do run $v c5 10 2 1 || exit 1; done
