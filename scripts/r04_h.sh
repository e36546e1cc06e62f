#!/bin/bash
# Round 4: counters of the kernels matching KRE (default k_score_wave|k_df_hist_lds|k_tokcount)
# on CFG (default c2), one rocprofv3 --pmc pass per counter group, then a kernel trace;
# summaries per kernel.  MODE: TFIDF_K1 value (default: the library's own choice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${TAG:-r04h}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
KRE=${KRE:-"k_score_wave|k_df_hist_lds|k_tokcount"}
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config ${CFG:-c2}"
[ -n "$MODE" ] && export TFIDF_K1=$MODE
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $CMD > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 1; }
for k in $(echo $KRE | tr '|' ' '); do echo "== $k"; python3 $R/scripts/pmc_summary.py $OUT $k; done
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -25 "$f" | cut -c1-160
