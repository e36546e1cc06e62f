#!/bin/bash
# Round 5: c2 kernel trace (csv) for the per-run timeline (scripts/timeline.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05tl
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe ${ARGS} > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 1; }
echo "trace done"
