#!/bin/bash
# K1 diagnosis pass (GPU box), every GPU step under its own limit, stops at the first failure:
#   phase stamps (lib/libtfidf_hip_stamps.so), timing-only ablations (lib/libtfidf_hip_s<N>.so),
#   the PMC passes of prof_k1.sh and the traffic entry.  Libraries are built in the dev container.
#   CFG=c2 bash scripts/diag_k1.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
T=${1:-diag}
CFG=${CFG:-c2}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
if [ "${STAMPS:-1}" = 1 ]; then
  TFIDF_LIB=stamps TFIDF_STAMPS=1 timeout -k 10 200 python3 -u scripts/k1_stamps.py $CFG > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -5 $OUT/stamps.txt; exit 1; }
  cat $OUT/stamps.txt
fi
for v in base ${VARIANTS:-}; do
  if [ "$v" = base ]; then lib=""; abl=""; else lib=$v; abl=1; fi
  TFIDF_LIB=$lib TFIDF_K1_ABLATE=$abl timeout -k 10 200 python3 -u bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-probe --no-emit > $OUT/abl_$v.json 2> $OUT/abl_$v.err || { echo "$v failed"; tail -5 $OUT/abl_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/abl_$v.json'));print('$v', 'K1 ms', d['roofline']['k1_avg_ms'])"
done
if [ "${PMC:-1}" = 1 ]; then
  BENCH_ARGS="--config $CFG" bash scripts/prof_k1.sh ${T}_$CFG > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${T}_$CFG k_tokcount_st > $OUT/pmc_summary.txt 2>&1
  cat $OUT/pmc_summary.txt
  python3 scripts/traffic_k1.py gpurun_out/prof_${T}_$CFG $CFG $OUT/k1_pmc_traffic.json
fi
