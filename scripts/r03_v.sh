#!/bin/bash
# Round 3: K1 chunk size (CHUNK_BYTES 12/16/24/32 KiB; 32 KiB also with 8-slot LDS
# buckets): per-chunk overhead (set-up, flush, barrier wait, chunk end) vs table load.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03w}
mkdir -p $OUT
for rep in 1 2 3; do
for cfg in c2 c5; do
for v in default ch20 ch24 ch24b8; do
  if [ $v = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$v; fi
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));s=d['stage_ms_mean'];print('$cfg $v', d['value'], d['ms_per_step'], s['tokcount'], s['merge'], s['df'], s['score'])"
done
done
done
