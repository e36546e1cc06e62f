#!/bin/bash
# Instruction counts of K1 ablation builds (one SQ counter pass per build, bench's K1 only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/ablpmc
mkdir -p $OUT
for v in base ${VARIANTS:-s1 s2 s4 s8}; do
  if [ "$v" = base ]; then lib=""; abl=""; else lib=$v; abl=1; fi
  TFIDF_LIB=$lib TFIDF_K1_ABLATE=$abl timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --kernel-include-regex k_tokcount --output-format csv -d $OUT/$v -o $v -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.log; exit 1; }
  echo "== $v"; python3 $R/scripts/pmc_summary.py $OUT/$v k_tokcount
done
