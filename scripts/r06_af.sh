#!/bin/bash
# c4: vocabulary table load limit past 16M slots (TFIDF_VLOAD_BIG): 45 (default: 32M slots,
# 512 MB of keys) against 65 / 80 (16M slots, 256 MB: the size of the MALL)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06af
mkdir -p $OUT
cd $R
run() {   # load tag
  TFIDF_VLOAD_BIG=$1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config c4 --steps 5 --warmup 2 > $OUT/c4_$1_$2.json 2> $OUT/c4_$1_$2.err || { echo "bench $1 failed"; tail -5 $OUT/c4_$1_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$1_$2.json')); print('c4 load $1', d['value'], d['ms_per_step'], 'k1', d['roofline']['k1_avg_ms'], d['stage_ms_mean'], d.get('k1_work',{}).get('partial_records'))"
}
for rnd in 1 2 3; do
  for l in 45 65 80; do run $l $rnd || exit 1; done
done
