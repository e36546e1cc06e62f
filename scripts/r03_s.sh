#!/bin/bash
# Round 3: candidate build (non-temporal DF and K5 record streams, word-store emission)
# vs DF-only non-temporal (ntdf) and the product build: full GPU tests on the candidate,
# then c4 / c2 A/B with the emission measurement on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03s}
mkdir -p $OUT
# on the box's scratch copy only: the candidate becomes the library the CLI links, the
# product build stays selectable as TFIDF_LIB=prod
L=parallel-systems-mpi-tfidf_amd/lib
cp $L/libtfidf_hip.so $L/libtfidf_hip_prod.so && cp $L/libtfidf_hip_cand.so $L/libtfidf_hip.so || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests_cand.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests_cand.log; exit 1; }
echo "cand gpu tests: $(tail -1 $OUT/gpu_tests_cand.log)"
for rep in 1 2; do
for cfg in c4 c2; do
for v in cand ntdf prod; do
  if [ $v = cand ]; then unset TFIDF_LIB; else export TFIDF_LIB=$v; fi
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));print('$cfg $v', d['value'], d['ms_per_step'], d['stage_ms_mean']['df'], d['stage_ms_mean']['score'], d['emit']['format_ms'])"
done
done
done
