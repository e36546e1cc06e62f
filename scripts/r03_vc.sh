#!/bin/bash
# Round 3: c2 / c5 vocabulary table size (TFIDF_VCAP initial slots; default 1M at <= 12 %
# load): K1's two-slot probes hit L2 more often in a smaller table, displace more keys.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03vc}
mkdir -p $OUT
run() {  # cfg vcap vload rep
  timeout -k 10 300 env TFIDF_VCAP=$2 TFIDF_VLOAD=$3 python3 -u bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_$1_$2_$4.json 2> $OUT/bench_$1_$2_$4.err \
      || { echo "bench $1 $2 failed"; tail -5 $OUT/bench_$1_$2_$4.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$1_$2_$4.json'));s=d['stage_ms_mean'];print('$1 vcap $2', d['value'], d['ms_per_step'], s['tokcount'], s['vocab'], s['df'], s['score'], d['k1_work']['vocab_capacity'], d['k1_work']['partial_records'])"
}
for rep in 1 2; do
  for cfg in c2 c5; do
    run $cfg 1048576 12 $rep || exit 1
    run $cfg 524288 12 $rep || exit 1
    run $cfg 262144 25 $rep || exit 1
    run $cfg 2097152 12 $rep || exit 1
  done
done
