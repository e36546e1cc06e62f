#!/bin/bash
# Round 5: kernel trace of config 3 on one GPU (rocpd database -> scripts/rocpd_stats.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05t
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/${CFG:-c3} -o run -- python3 bench.py --config ${CFG:-c3} --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/${CFG:-c3}.json 2> $OUT/${CFG:-c3}.err || { tail -20 $OUT/${CFG:-c3}.err; exit 1; }
db=$(find $OUT/${CFG:-c3} -name "*.db" | head -1)
python3 scripts/rocpd_stats.py $db 30 > $OUT/${CFG:-c3}_kernel_stats.csv && cat $OUT/${CFG:-c3}_kernel_stats.csv
