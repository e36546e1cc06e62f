#!/bin/bash
# Round 5: kernel traces of config 4 (one shard, then 8 shards on the GPU: the hash-owner DF
# exchange) for the DF / exchange breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05f
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
echo "c4 done"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c4x8 -o run -- python3 bench.py --config c4 --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $OUT/c4x8.json 2> $OUT/c4x8.err || { tail -20 $OUT/c4x8.err; exit 1; }
echo "c4x8 done"
for d in c4 c4x8; do
  f=$(find $OUT/$d -name "*kernel_stats.csv" | sort | tail -1)
  [ -n "$f" ] && cp $f $OUT/${d}_kernel_stats.csv && python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/${d}_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:30]: print('$d', r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs'])/1e6,3), round(float(r['AverageNs'])/1e3,1))
"
done
