#!/bin/bash
# Round 3: owner exchange with claim-counted inserts and a 1.5x table — multi-rank parity,
# the 8-shard exchange (c4/c5), the c2 kernel-trace stats + K1 PMC traffic (c2, c5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03k}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > $OUT/multirank.log 2>&1 \
    || { echo "multirank failed"; tail -30 $OUT/multirank.log; exit 1; }
tail -1 $OUT/multirank.log
for cfg in c5 c4; do
  timeout -k 10 400 python3 -u bench.py --config $cfg --shards 8 --steps 3 --warmup 1 > $OUT/shards8_$cfg.json 2> $OUT/shards8_$cfg.err || { echo "shards $cfg failed"; tail -20 $OUT/shards8_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/shards8_$cfg.json'));print('$cfg x8', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_frac_of_step'], d['nterms_global'], d['stage_ms_max_over_ranks_mean'])"
done
CFGS="c2 c5" STEPS=10 bash scripts/measure_cfgs.sh r03k_cfgs || exit 1
