#!/bin/bash
# K1 memory-pipeline and LDS counters, one rocprofv3 --pmc pass per group (GPU box):
#   bash scripts/prof_k1_mem.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-mem}
OUT=$R/gpurun_out/prof_$T
mkdir -p $OUT
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for pmc in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_tokcount" --output-format csv -d $OUT/m$i -o m$i -- $CMD > $OUT/m$i.log 2>&1
done
python3 - $OUT <<'PY'
import csv, glob, collections, sys
for f in sorted(glob.glob(sys.argv[1] + "/m*/m*_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_tokcount" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(k, "%.4g" % v[-1])
PY
