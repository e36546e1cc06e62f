#!/bin/bash
# Round 5: baseline of the round-4 tree on a fresh box: c2 bench x2, K1 phase stamps (c2), c4 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05base
mkdir -p $OUT
cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { tail -20 $OUT/bench_c2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
done
TFIDF_LIB=stamps TFIDF_STAMPS=1 timeout -k 10 300 python3 scripts/k1_stamps.py c2 > $OUT/stamps_c2.txt 2>&1 || { tail -20 $OUT/stamps_c2.txt; exit 1; }
cat $OUT/stamps_c2.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c4 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['stage_ms_mean'])"
