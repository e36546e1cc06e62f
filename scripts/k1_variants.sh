#!/bin/bash
# Full-pipeline A/B of prebuilt library variants (lib/libtfidf_hip_<name>.so, built here with
# `make variant NAME=<name> DEFS=...`) against the default build, on one config; each variant
# is also checked against the oracle (the synthetic-config parity tests) unless CHECK=0.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/var
timeout -k 10 600 make -j16 -C parallel-systems-mpi-tfidf_amd > gpurun_out/make.log 2>&1 || { echo "make failed"; tail -30 gpurun_out/make.log; exit 1; }
for v in base ${VARIANTS}; do
  lib=$v; [ "$v" = base ] && lib=""
  TFIDF_LIB=$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-probe --no-emit ${BENCH_ARGS:-} > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { echo "$v bench failed"; tail -5 gpurun_out/var/$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var/$v.json'));print('$v', d['value'], 'K1 ms', d['roofline']['k1_avg_ms'], d['k1_work'], d['stage_ms'])"
  if [ "${CHECK:-1}" = 1 ] && { [ "$v" != base ] || [ "${CHECK_BASE:-0}" = 1 ]; }; then
    TFIDF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${CHECK_SEL:-synthetic_configs or big_docs or many_tiny or more_pairs or nul or long_tokens or boundaries or empty or across}" > gpurun_out/var/$v.test.log 2>&1 || { echo "$v parity failed"; tail -15 gpurun_out/var/$v.test.log; exit 1; }
    tail -1 gpurun_out/var/$v.test.log
  fi
done
