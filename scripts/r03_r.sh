#!/bin/bash
# Round 3: non-temporal record streams in the large-V DF kernels (ntdf) vs the product
# build: parity at c4 scale, c4 and c2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03r}
mkdir -p $OUT
TFIDF_LIB=ntk5 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "full_config or synthetic or variants" > $OUT/parity_ntk5.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity_ntk5.log; exit 1; }
echo "ntk5 parity: $(tail -1 $OUT/parity_ntk5.log)"
for rep in 1 2; do
for cfg in c4 c2; do
for v in ntk5 ntdf default; do
  if [ $v = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$v; fi
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));print('$cfg $v', d['value'], d['ms_per_step'], d['stage_ms_mean']['df'], d['stage_ms_mean']['score'])"
done
done
done
