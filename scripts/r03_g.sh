#!/bin/bash
# Round 3: product library (k_tokcount_st default) — default bench as the first GPU process,
# hip-trace of a fresh-process bench (allocations between timed steps), c3/c4/c5 lines,
# the DF exchange at 8 shards on one GPU (c3/c4/c5), then every GPU test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03g}
mkdir -p $OUT
echo "== default bench (first GPU process of the box)"
timeout -k 10 400 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['cold_run_ms'], d['cpu_baseline']['value'])"
echo "== hip trace"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/hiptrace -o t -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-probe > $OUT/hiptrace_bench.json 2> $OUT/hiptrace.err ) || { echo "hip trace failed"; tail -20 $OUT/hiptrace.err; exit 1; }
python3 scripts/alloc_trace.py $OUT/hiptrace 2 10 || true
for cfg in c4 c5; do
  echo "== $cfg"
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['stage_ms_mean'])"
done
echo "== c3 (40 GB, 1 GPU)"
timeout -k 10 400 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -20 $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
for cfg in c5 c4 c3; do
  echo "== $cfg x 8 shards"
  timeout -k 10 400 python3 -u bench.py --config $cfg --shards 8 --steps 3 --warmup 1 > $OUT/shards8_$cfg.json 2> $OUT/shards8_$cfg.err || { echo "shards $cfg failed"; tail -20 $OUT/shards8_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/shards8_$cfg.json'));print('$cfg x8', d['value'], d['ms_per_step'], d['exchange_ms'], d['exchange_frac_of_step'], d['stage_ms_max_over_ranks_mean'])"
done
echo "== GPU tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
