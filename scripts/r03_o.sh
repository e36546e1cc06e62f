#!/bin/bash
# Round 3: the tree as it stands — every GPU test, then the default bench and c4/c5 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03o}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print('c2', d['value'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['device_allocs_in_timed_steps'], d['stage_ms_mean'])"
for cfg in c5 c4; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['stage_ms_mean'])"
done
