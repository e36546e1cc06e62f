#!/bin/bash
# Round 4, call D: K1 counters, sl vs st (one rocprofv3 --pmc pass per counter group)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04d
mkdir -p $OUT
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe"
for k in sl st; do
  i=0
  for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
             "SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH SQ_INSTS_SENDMSG" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    TFIDF_K1=$k timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/${k}_p$i -o p$i -- $CMD > $OUT/${k}_p$i.log 2>&1 || { echo "pass $k $i failed"; tail -5 $OUT/${k}_p$i.log; }
  done
done
for k in sl st; do echo "== $k"; python3 $R/scripts/pmc_summary.py $OUT k_tokcount_$k; done
