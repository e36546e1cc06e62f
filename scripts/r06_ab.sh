#!/bin/bash
# c4 at 8 shards on one GPU: kernel trace of the exchange (which kernels of which rank run when)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config c4 > $OUT/shards8_c4.json 2> $OUT/shards8_c4.err || { echo "trace failed"; tail -5 $OUT/shards8_c4.err; exit 1; }
echo "shards8 c4: $(tail -1 $OUT/shards8_c4.json | cut -c1-600)"
F=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/xchg_timeline.py $F > $OUT/xchg_timeline.txt && tail -80 $OUT/xchg_timeline.txt
