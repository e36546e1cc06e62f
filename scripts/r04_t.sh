#!/bin/bash
# Round 4: K1 HBM traffic per config (FETCH_SIZE and WRITE_SIZE passes, one rocprofv3 run
# each) for scripts/traffic_k1.py -> profiles/k1_pmc_traffic.json.  CFGS (default c2 c4 c5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for c in ${CFGS:-c2 c4 c5}; do
  OUT=$R/gpurun_out/r04t_$c
  mkdir -p $OUT
  CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config $c"
  i=0
  for pmc in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $c $pmc failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  echo "$c done"
done
