#!/bin/bash
# Round 5: 8 shards on one GPU with the HIP runtime's hardware queues per process at the
# box default (4: the 8 ranks' 16 streams share them) and at 16 (one per stream).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05q
mkdir -p $OUT
cd $R
for q in default 16 default 16; do
  for c in c5 c4; do
    EV=""; [ $q != default ] && EV="GPU_MAX_HW_QUEUES=$q"
    env $EV timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/q${q}_$c.json 2> $OUT/q${q}_$c.err || { echo "fail $q $c"; tail -5 $OUT/q${q}_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/q${q}_$c.json')); s=d['stage_ms_max_over_ranks_mean']; print('$q $c', d['value'], d['ms_per_step'], d['exchange_ms_min_over_ranks'], 'idf', s['idf'], 'order', s['order'], 'exch', s['exchange'])"
  done
done
