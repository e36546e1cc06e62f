#!/bin/bash
# Round 3: product build (carried-chunk emission, plain K5 stores, DF non-temporal record
# streams): all GPU tests, default bench, c4 vocabulary load limit 45 % vs 60 %
# (TFIDF_VLOAD_BIG: 32M vs 16M slots), kernel stats of a c2 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03u}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
for rep in 1 2; do
for vl in 45 60; do
  TFIDF_VLOAD_BIG=$vl timeout -k 10 300 python3 -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $OUT/bench_c4_vl${vl}_$rep.json 2> $OUT/bench_c4_vl${vl}_$rep.err \
      || { echo "bench c4 $vl failed"; tail -5 $OUT/bench_c4_vl${vl}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_c4_vl${vl}_$rep.json'));print('c4 vload $vl', d['value'], d['ms_per_step'], d['stage_ms_mean'], d['emit']['format_ms'])"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $OUT/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_c2.log; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_c2.csv
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/kernel_stats_c2.csv')))
for x in r[:24]: print(x['Name'][:60], x['Calls'], x['AverageNs'])
"
