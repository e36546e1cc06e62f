#!/bin/bash
# Round measurement set (GPU box), every step under its own time limit:
#   1. K1 PMC passes (rocprofv3 --pmc, one pass per counter group) -> HBM traffic per launch
#   2. rocprofv3 --kernel-trace --stats of a short bench run        -> per-kernel averages
#   3. the default bench line (with the CPU baseline)              -> bench JSON
# Results land in gpurun_out/<tag>/ (copied into profiles/ by hand and committed).
#   bash scripts/measure_round.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-round}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
bash $R/scripts/prof_k1.sh $T > $OUT/pmc.log 2>&1
python3 $R/scripts/traffic_k1.py $R/gpurun_out/prof_$T ${KEY:-c2} $OUT/k1_pmc_traffic.json
bash $R/scripts/kstats.sh $T > $OUT/kernel_stats.txt 2>&1
cp $(find $R/gpurun_out/ks_$T -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
cd $R && timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
