#!/bin/bash
# Round 3: DF histogram workgroups balanced to whole CU waves (dft) and, on top of it,
# branch-free vocabulary hit compares in K1 (hx) vs the product build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03dh}
mkdir -p $OUT
TFIDF_LIB=hx timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "not cli" > $OUT/parity_hx.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity_hx.log; exit 1; }
echo "hx parity: $(tail -1 $OUT/parity_hx.log)"
run() {  # cfg variant rep
  if [ $2 = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$2; fi
  timeout -k 10 300 python3 -u bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_$1_$2_$3.json 2> $OUT/bench_$1_$2_$3.err \
      || { echo "bench $1 $2 failed"; tail -5 $OUT/bench_$1_$2_$3.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$1_$2_$3.json'));s=d['stage_ms_mean'];print('$1 $2', d['value'], d['ms_per_step'], s['tokcount'], s['merge'], s['df'], s['score'])"
}
for rep in 1 2 3; do
  for cfg in c2 c5; do for v in default dft hx; do run $cfg $v $rep || exit 1; done; done
done
