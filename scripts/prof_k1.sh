#!/bin/bash
# K1 counter passes (one rocprofv3 --pmc pass per counter group, each under its own
# time limit).  Usage (GPU box): bash scripts/prof_k1.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-k1}
OUT=$R/gpurun_out/prof_$T
mkdir -p $OUT
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe ${BENCH_ARGS:-}"
PASSES=${PASSES:-5}
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "${KREGEX:-k_tokcount}" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $CMD > $OUT/kt.log 2>&1
find $OUT -name "*.csv" | head -50
