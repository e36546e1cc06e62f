#!/bin/bash
# Round 3, final tree: single-GPU lines of c3 / c4 / c5 and the 8-shard (one GPU,
# in-process exchange) lines of c3 / c4 / c5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03cfgs}
mkdir -p $OUT
for cfg in c5 c4; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -5 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['stage_ms_mean'], d['roofline']['frac'], d['roofline']['traffic'])"
done
timeout -k 10 600 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -5 $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', d['value'], d['ms_per_step'], d['stage_ms_mean'])"
for cfg in c3 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $cfg --shards 8 --steps 3 --warmup 1 > $OUT/shards8_$cfg.json 2> $OUT/shards8_$cfg.err || { echo "shards $cfg failed"; tail -20 $OUT/shards8_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/shards8_$cfg.json'));print('$cfg x8', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_frac_of_step'])"
done
