#!/bin/bash
# Kernel timeline of one pipeline run (GPU box): every kernel of the last run and the idle
# gaps between them, to find host round trips between stages.   CFG=c2 bash scripts/gap_timeline.sh
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${CFG:-c2}
timeout -s KILL 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/gap_$C -o gap -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/gap_$C.log 2>&1 || { tail -5 $R/gpurun_out/gap_$C.log; exit 1; }
python3 - $R/gpurun_out/gap_$C <<'PY'
import csv, sys, glob
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in csv.DictReader(open(f))]
for f in glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")) for r in csv.DictReader(open(f))]
rows.sort()
ks = [i for i, r in enumerate(rows) if "tokcount" in r[2]]
i0 = max(ks[-1] - 8, 0) if ks else 0
t0 = rows[i0][0]
end = rows[i0][0]
for s, e, n in rows[i0:]:
    print("%9.1f us  gap %7.1f  dur %7.1f  %s" % ((s - t0) / 1e3, (s - end) / 1e3, (e - s) / 1e3, n))
    end = max(end, e)
PY
