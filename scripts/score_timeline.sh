cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_${CFG:-c4} -o tl -- python3 $R/bench.py --config ${CFG:-c4} --steps 2 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/tl_${CFG:-c4}.log 2>&1 || { tail -5 $R/gpurun_out/tl_${CFG:-c4}.log; exit 1; }
python3 - $(find $R/gpurun_out/tl_${CFG:-c4} -name "*kernel_trace.csv" | head -1) <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'k_score_wave' in r['Kernel_Name']]
i0=idx[-1]-7
t0=int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i0+14]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    print("%8.1f us  dur %7.1f  q%s %s"%((s-t0)/1e3,(e-s)/1e3,r['Queue_Id'],r['Kernel_Name'][:50]))
PY
