#!/bin/bash
# Round 3: tokcount_st overflow margin (fill limit TB - 320 instead of TB - 576), with 24
# and 28 KiB chunks; tokcount_vs (c4) with 24 KiB chunks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03y}
mkdir -p $OUT
run() {  # cfg variant rep
  if [ $2 = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$2; fi
  timeout -k 10 300 python3 -u bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_$1_$2_$3.json 2> $OUT/bench_$1_$2_$3.err \
      || { echo "bench $1 $2 failed"; tail -5 $OUT/bench_$1_$2_$3.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$1_$2_$3.json'));s=d['stage_ms_mean'];print('$1 $2', d['value'], d['ms_per_step'], s['tokcount'], s['merge'], s['df'], s['score'])"
}
for rep in 1 2; do
  for cfg in c2 c5; do for v in default fl fl28; do run $cfg $v $rep || exit 1; done; done
  for v in default vs24; do run c4 $v $rep || exit 1; done
done
