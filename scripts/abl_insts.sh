#!/bin/bash
# Dynamic instruction counts of K1 per ablation build (GPU box): one rocprofv3 --pmc pass
# per ablation (lib/libtfidf_hip_abl<N>.so), then the per-dispatch medians.
#   ABL="0 1 2 16 64 128" bash scripts/abl_insts.sh
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for a in ${ABL:-0}; do
  if [ "$a" = "0" ]; then V=""; else V="abl$a"; fi
  OUT=$R/gpurun_out/ai_$a
  TFIDF_LIB=$V TFIDF_K1_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
      --kernel-include-regex k_tokcount --output-format csv -d $OUT/p1 -o p1 -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT.log 2>&1 || exit 1
  echo "== abl $a"; python3 $R/scripts/pmc_summary.py $OUT k_tokcount
done
