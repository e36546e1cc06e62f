#!/bin/bash
# Round 6 Q: K5 emission batch size with the compile-time idf path (k5eN: N idf gathers per
# lane in flight, 2 VGPRs spilled; default N = 8: 15 spilled) against the committed kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06q
mkdir -p $OUT
cd $R
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'score', s['score'], 'df', s['df'], 'merge', s['merge'])"
}
for rnd in 1 2; do
  for v in k5head k5e1 k5e2 k5e4 default; do run $v c2 20 3 $rnd || exit 1; done
done
for v in k5head k5e1 k5e2 k5e4; do run $v c3 3 1 1 || exit 1; done
