set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/split_debug.py g5_w1 g4_config1 > gpurun_out/diff.txt 2>&1 || { cat gpurun_out/diff.txt; exit 1; }
cat gpurun_out/diff.txt
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_split -o ks -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-emit --no-probe > gpurun_out/ks_bench.json 2>gpurun_out/ks.err || { tail gpurun_out/ks.err; exit 1; }
find gpurun_out/ks_split -name "*kernel_stats.csv" | head -1 | xargs head -14
