#!/bin/bash
# Round-2 final measurement set (GPU box): default c2 bench line with the CPU baseline,
# kernel-trace stats of c2, c4, c5 bench lines (the K1 PMC traffic entries of
# profiles/k1_pmc_traffic.json stay valid: their K1 sources are unchanged).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r02_final
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -5 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
bash scripts/kstats.sh r02f_c2 > $OUT/kernel_stats_c2.txt 2>&1 || { echo "kstats failed"; exit 1; }
head -8 $OUT/kernel_stats_c2.txt
KSTATS=0 PMC=0 CFGS="c4 c5" bash scripts/measure_cfgs.sh r02_final || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -20 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
