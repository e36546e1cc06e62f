#!/bin/bash
# Round 4, call B: the one-workgroup-per-chunk K1 (k_tokcount_sl) as the default: GPU tests,
# smoke, bench c2 (sl vs the persistent st kernel), kernel trace of the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04b
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
for k in sl st sl st; do
  TFIDF_K1=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 20 --warmup 3 > $OUT/bench_$k.json 2>> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$k.json')); print('$k', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --no-emit > $OUT/ks.log 2>&1 || { tail $OUT/ks.log; exit 1; }
f=$(find $OUT/ks -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv | cut -d, -f1-8
