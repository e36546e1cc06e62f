#!/bin/bash
# Round 3: k_tokcount_st at 3 workgroups per CU (151 VGPRs, no VGPR spills) with the
# default and a 5120-entry table, against the product build (4 per CU): parity, c2/c5 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03p}
mkdir -p $OUT
for v in wg3 wg3t5; do
  TFIDF_LIB=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "golden or synthetic or big_docs or more_pairs or tiny or boundaries or dense_merge or variants" > $OUT/parity_$v.log 2>&1 \
      || { echo "parity $v failed"; tail -30 $OUT/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $OUT/parity_$v.log)"
done
for rep in 1 2; do
for cfg in c2 c5; do
for v in wg3 wg3t5 default; do
  if [ $v = default ]; then unset TFIDF_LIB; else export TFIDF_LIB=$v; fi
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));print('$cfg $v', d['value'], d['roofline']['k1_avg_ms'], d['k1_work']['partial_records'], d['stage_ms_mean']['merge'], d['ms_per_step'])"
done
done
done
