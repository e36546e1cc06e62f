#!/bin/bash
# K1 ablation timings (timing-only builds lib/libtfidf_hip_s<N>.so, built in the dev
# container: make variant NAME=sN DEFS=-DK1S_ABL=N) + two SQ counter passes of the default K1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/abl
timeout -k 10 600 make -j16 -C parallel-systems-mpi-tfidf_amd > gpurun_out/make.log 2>&1 || { echo "make failed"; exit 1; }
for v in base ${VARIANTS:-s1 s2 s4 s8 s16}; do
  if [ "$v" = base ]; then lib=""; abl=""; else lib=$v; abl=1; fi
  TFIDF_LIB=$lib TFIDF_K1_ABLATE=$abl timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-probe --no-emit ${BENCH_ARGS:-} > gpurun_out/abl/$v.json 2> gpurun_out/abl/$v.err || { echo "$v failed"; tail -5 gpurun_out/abl/$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abl/$v.json'));print('$v', 'K1 ms', d['roofline']['k1_avg_ms'])"
done
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  OUT=$R/gpurun_out/abl/pmc
  mkdir -p $OUT
  i=0
  for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex k_tokcount --output-format csv -d $OUT/p$i -o p$i -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  done
  python3 $R/scripts/pmc_summary.py $OUT k_tokcount
fi
