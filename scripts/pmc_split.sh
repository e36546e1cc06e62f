#!/bin/bash
# SQ counter passes for the split K1 kernels (GPU box), one rocprofv3 --pmc pass per group.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-split}
OUT=$R/gpurun_out/pmc_$T
mkdir -p $OUT
CMD="python3 $R/bench.py --config ${CFG:-c2} --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "${KREGEX:-k_tok_resolve|k_count_slots}" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
for k in ${KNAMES:-k_tok_resolve k_count_slots}; do echo "== $k"; python3 $R/scripts/pmc_summary.py $OUT $k; done
