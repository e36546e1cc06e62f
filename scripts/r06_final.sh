#!/bin/bash
# Round 6 final measurement of the committed tree, part PART:
#   1: full GPU suite, smoke, the driver's default bench (c2) x3, c3/c4/c5 benches, 8-shard exchange benches
#   2: K1 counters on c2 (SQ groups, FETCH/WRITE) -> profiles/r06_k1_pmc_c2.txt, K1 traffic per config
#      (c2 c3 c4 c5, and rank 0's shard of the multi-GPU plans: c2 weak g2/g4/g8, c3 strong g8), c2 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06final
mkdir -p $OUT
cd $R
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; tail -3 $OUT/gpu_tests.log; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
  echo "smoke: $(tail -1 $OUT/smoke.log)"
  for i in 1 2 3; do
    timeout -k 10 600 python3 bench.py > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { echo "bench failed"; tail -20 $OUT/bench_c2_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['stage_ms_mean'])"
  done
  for c in c3 c4 c5; do
    timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
  done
  for c in c5 c3 c4; do
    timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
    echo "shards8 $c: $(tail -1 $OUT/shards8_$c.json | cut -c1-240)"
  done
else
  cd /tmp && export TMPDIR=/tmp
  CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config c2"
  i=0
  for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount|k_score_wave|k_score_fill|k_df_hist_lds" --output-format csv -d $OUT/pmc_c2/p$i -o p$i -- $CMD > $OUT/pmc_c2_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_c2_p$i.log; exit 1; }
  done
  echo "pmc c2 done"
  run_traffic() {   # name, bench args
    local n=$1; shift
    local j=0
    for pmc in FETCH_SIZE WRITE_SIZE; do
      j=$((j+1))
      timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/traffic_$n/p$j -o p$j -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe "$@" > $OUT/traffic_${n}_p$j.log 2>&1 || { echo "traffic $n $pmc failed"; tail -5 $OUT/traffic_${n}_p$j.log; return 1; }
    done
    echo "traffic $n done"
  }
  if [ "${SKIP_TRAFFIC:-0}" != 1 ]; then   # SKIP_TRAFFIC=1: counters and trace only (K1 unchanged)
  run_traffic c2 --config c2 && run_traffic c4 --config c4 && run_traffic c5 --config c5 && \
  run_traffic c2_g2 --config c2 --shard-of 0/2 && run_traffic c2_g4 --config c2 --shard-of 0/4 && \
  run_traffic c2_g8 --config c2 --shard-of 0/8 && run_traffic c3 --config c3 && run_traffic c3_strong_g8 --config c3 --strong --shard-of 0/8 || exit 1
  fi
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c2 -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/kt_c2.log 2>&1 || { echo "trace failed"; exit 1; }
  echo "trace done"
fi
