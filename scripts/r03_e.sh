#!/bin/bash
# Round 3: K1 variant check — quick parity, A/B bench (lean vs st), lean counters, GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03e}
mkdir -p $OUT
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "golden or variants or edge or boundaries or big_docs or classes" > $OUT/quick.log 2>&1 || { echo "quick parity failed"; tail -30 $OUT/quick.log; exit 1; }
tail -1 $OUT/quick.log
for v in lean st; do
  if [ $v = st ]; then export TFIDF_K1=st; else unset TFIDF_K1; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $OUT/bench_$v.json 2> $OUT/bench_$v.err \
      || { echo "bench $v failed"; tail -5 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['k1_work'])"
done
unset TFIDF_K1
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/pmc_lean_p$i -o p -- $CMD > $OUT/pmc_lean_p$i.log 2>&1 \
      || { echo "pmc $i failed"; tail -5 $OUT/pmc_lean_p$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $OUT/pmc_lean_p$i k_tokcount
done
cd $R
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
fi
