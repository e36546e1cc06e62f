#!/bin/bash
# Round 3: product build with 24 KiB tokcount_st chunks and 8-slot LDS buckets: all GPU
# tests, default bench, c5 / c4 / c3 lines, kernel stats and K1 traffic counters of c2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03x}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print('default', d['value'], d['ms_per_step'], d['stage_ms_mean'], d['roofline']['frac'])"
for cfg in c5 c4 c2; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -5 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['stage_ms_mean'])"
done
timeout -k 10 600 python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -5 $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', d['value'], d['ms_per_step'], d['stage_ms_mean'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $OUT/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_c2.log; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_c2.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_tokcount --output-format csv -d $OUT/pmc_fetch -o f -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_tokcount --output-format csv -d $OUT/pmc_write -o w -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $OUT/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS --kernel-include-regex k_tokcount --output-format csv -d $OUT/pmc_sq -o s -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 $OUT/pmc_sq.log; exit 1; }
echo done
