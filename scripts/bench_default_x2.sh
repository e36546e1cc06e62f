#!/bin/bash
# The driver's default bench command, twice, then once with per-step device timings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bd
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py > gpurun_out/bd/b$i.json 2> gpurun_out/bd/b$i.err || { echo "bench $i failed"; tail -5 gpurun_out/bd/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bd/b$i.json')); print($i, d['value'], d['ms_per_step'], d['device_ms_per_step'], d['stage_ms']['score'], d['roofline']['traffic'])"
done
