#!/bin/bash
# Per-config measurement set (GPU box): bench line, kernel-trace stats and the K1 PMC
# passes (traffic entry) for each config in CFGS.  Every GPU step has its own limit; the
# chain stops at the first failure.   CFGS="c4 c5" bash scripts/measure_cfgs.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
T=${1:-cfgs}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
for cfg in ${CFGS:-c4 c5}; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-probe > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -5 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], 'GB/s', d['ms_per_step'], 'ms/step K1', d['roofline']['k1_avg_ms'], d['k1_work'], d['stage_ms'])"
  if [ "${KSTATS:-1}" = 1 ]; then
    bash scripts/kstats.sh ${T}_$cfg --config $cfg > $OUT/kernel_stats_$cfg.txt 2>&1 || { echo "kstats $cfg failed"; tail -5 $OUT/kernel_stats_$cfg.txt; exit 1; }
    head -12 $OUT/kernel_stats_$cfg.txt
  fi
  if [ "${PMC:-1}" = 1 ]; then
    PASSES=5 BENCH_ARGS="--config $cfg" bash scripts/prof_k1.sh ${T}_$cfg > $OUT/pmc_$cfg.log 2>&1 || { echo "pmc $cfg failed"; tail -5 $OUT/pmc_$cfg.log; exit 1; }
    python3 scripts/pmc_summary.py gpurun_out/prof_${T}_$cfg k_tokcount_st > $OUT/pmc_summary_$cfg.txt 2>&1
    python3 scripts/traffic_k1.py gpurun_out/prof_${T}_$cfg $cfg $OUT/k1_pmc_traffic_$cfg.json
  fi
done
