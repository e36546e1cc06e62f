#!/bin/bash
# Round 3: K5 with non-temporal record loads only (k5ld) vs DF-only (ntdf) and the
# candidate with non-temporal K5 stores too (cand); kernel stats of the emission kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03t}
mkdir -p $OUT
TFIDF_LIB=k5ld timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "full_config or synthetic or variants" > $OUT/parity_k5ld.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity_k5ld.log; exit 1; }
echo "k5ld parity: $(tail -1 $OUT/parity_k5ld.log)"
for rep in 1 2; do
for cfg in c4 c2; do
for v in k5ld ntdf cand; do
  export TFIDF_LIB=$v
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));print('$cfg $v', d['value'], d['ms_per_step'], d['stage_ms_mean']['df'], d['stage_ms_mean']['score'], d['emit']['format_ms'])"
done
done
done
export TFIDF_LIB=k5ld
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $OUT/prof_c2.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_c2.log; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_c2_k5ld.csv
head -30 $OUT/kernel_stats_c2_k5ld.csv | cut -c1-160
