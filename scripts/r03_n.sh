#!/bin/bash
# Round 3: k_tokcount_st scalar-register variants — k1o (output block through device memory,
# the product build), st2 (every argument but the per-step ones through device memory),
# prev (round-2 arguments): parity of both new ones, c2/c5 A/B, st2 counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03n}
mkdir -p $OUT
for v in k1o st2; do
  TFIDF_LIB=$v timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread \
      -k "not full_config" > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -40 $OUT/parity_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/parity_$v.log)"
done
for rep in 1 2; do
for cfg in c2 c5; do
for v in st2 k1o prev; do
  export TFIDF_LIB=$v
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_${cfg}_${v}_$rep.json 2> $OUT/bench_${cfg}_${v}_$rep.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_${v}_$rep.json'));print('$cfg $v', d['value'], d['roofline']['k1_avg_ms'], d['device_allocs_in_timed_steps'], d['k1_work']['partial_records'])"
done
done
done
export TFIDF_LIB=st2
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/pmc_p$i -o p -- $CMD > $OUT/pmc_p$i.log 2>&1 \
      || { echo "pmc $i failed"; tail -5 $OUT/pmc_p$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $OUT/pmc_p$i k_tokcount
done
