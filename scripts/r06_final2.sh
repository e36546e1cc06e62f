#!/bin/bash
# Round 6 final measurement of the committed tree (after the DF / K5 changes): full GPU suite,
# smoke, the driver's default bench (c2) x3, c3/c4/c5 benches, 8-shard exchange benches,
# c2 counters (K1 / K5 / DF), kernel traces of c2, c3 and c4.  K1 is unchanged since
# fa01436: its traffic entries (digest bba7c88...) stay valid.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06final2
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; tail -3 $OUT/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/gpu_tests.log)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { echo "bench failed"; tail -20 $OUT/bench_c2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['stage_ms_mean'])"
done
for c in c3 c4 c5; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['traffic'], d['stage_ms_mean'])"
done
for c in c5 c3 c4; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  echo "shards8 $c: $(tail -1 $OUT/shards8_$c.json | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config c2"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount|k_score_wave|k_score_small|k_df_hist_lds" --output-format csv -d $OUT/pmc_c2/p$i -o p$i -- $CMD > $OUT/pmc_c2_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_c2_p$i.log; exit 1; }
done
echo "pmc c2 done"
for c in c2 c3 c4; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config $c > $OUT/kt_$c.log 2>&1 || { echo "trace $c failed"; tail -5 $OUT/kt_$c.log; exit 1; }
  echo "trace $c done"
done
