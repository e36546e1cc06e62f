#!/bin/bash
# Round 3: windowed K1 — quick parity, c2/c5 bench A/B (win default vs lean vs st), win counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/${TAG:-r03f}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "not full_config" > $OUT/quick.log 2>&1 || { echo "quick parity failed"; tail -40 $OUT/quick.log; exit 1; }
tail -1 $OUT/quick.log
for cfg in c2 c5; do
for v in win lean st; do
  if [ $v = win ]; then unset TFIDF_K1; else export TFIDF_K1=$v; fi
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-emit > $OUT/bench_${cfg}_$v.json 2> $OUT/bench_${cfg}_$v.err \
      || { echo "bench $cfg $v failed"; tail -5 $OUT/bench_${cfg}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_$v.json'));print('$cfg $v', d['value'], d['roofline']['k1_avg_ms'], d['roofline']['kernel'], d['device_allocs_in_timed_steps'], d['k1_work'])"
done
done
unset TFIDF_K1
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/pmc_win_p$i -o p -- $CMD > $OUT/pmc_win_p$i.log 2>&1 \
      || { echo "pmc $i failed"; tail -5 $OUT/pmc_win_p$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $OUT/pmc_win_p$i k_tokcount
done
