#!/bin/bash
# Round 3: K1 with token entries carried across steps so that rounds run full (carry)
# vs the product build: parity on the K1 paths, then c2 / c5 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03z}
mkdir -p $OUT
TFIDF_LIB=carry timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "not cli" > $OUT/parity_carry.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity_carry.log; exit 1; }
echo "carry parity: $(tail -1 $OUT/parity_carry.log)"
run() {  # cfg variant rep
  if [ $2 = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$2; fi
  timeout -k 10 300 python3 -u bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_$1_$2_$3.json 2> $OUT/bench_$1_$2_$3.err \
      || { echo "bench $1 $2 failed"; tail -5 $OUT/bench_$1_$2_$3.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$1_$2_$3.json'));s=d['stage_ms_mean'];print('$1 $2', d['value'], d['ms_per_step'], s['tokcount'], s['merge'], s['df'], s['score'])"
}
for rep in 1 2; do
  for cfg in c2 c5; do for v in default carry; do run $cfg $v $rep || exit 1; done; done
done
