#!/bin/bash
# SQ instruction counters of K1 for the default build and the timing-only ablation builds
# (lib/libtfidf_hip_s<N>.so): where the VALU / SALU / LDS instructions go.  GPU box.
#   VARIANTS="s1 s2 s4 s64" bash scripts/abl_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-ablpmc}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
for v in base ${VARIANTS:-s1 s2 s4 s64}; do
  if [ "$v" = base ]; then lib=""; abl=""; else lib=$v; abl=1; fi
  TFIDF_LIB=$lib TFIDF_K1_ABLATE=$abl timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-include-regex k_tokcount --output-format csv -d $OUT/$v -o $v -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe ${BENCH_ARGS:-} > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.log; exit 1; }
  echo "== $v"; python3 $R/scripts/pmc_summary.py $OUT/$v k_tokcount
done
