#!/bin/bash
# Round 3: hash-owner exchange and the LDS-staged radix scatter — the DF exchange at 8
# shards on one GPU (c3/c4/c5), c4 and c5 single-GPU lines, the default bench, all GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03i}
mkdir -p $OUT
for cfg in c5 c4 c3; do
  echo "== $cfg x 8 shards"
  timeout -k 10 400 python3 -u bench.py --config $cfg --shards 8 --steps 3 --warmup 1 > $OUT/shards8_$cfg.json 2> $OUT/shards8_$cfg.err || { echo "shards $cfg failed"; tail -20 $OUT/shards8_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/shards8_$cfg.json'));print('$cfg x8', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_frac_of_step'], d['device_allocs_in_timed_steps'], d['stage_ms_max_over_ranks_mean'])"
done
for cfg in c4 c5; do
  echo "== $cfg"
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['stage_ms_mean'])"
done
echo "== default bench"
timeout -k 10 400 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['device_allocs_in_timed_steps'], d['cold_run_ms'], d['stage_ms_mean'])"
echo "== GPU tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
