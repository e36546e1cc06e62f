#!/bin/bash
# Round 3: c4 K1 (k_tokcount_vs) traffic counters for the current source (k1_pmc_traffic.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-r03pmc4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_tokcount --output-format csv -d $OUT/pmc4_fetch -o f -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/pmc4_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/pmc4_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_tokcount --output-format csv -d $OUT/pmc4_write -o w -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/pmc4_write.log 2>&1 || { echo "pmc write failed"; tail -5 $OUT/pmc4_write.log; exit 1; }
echo done
