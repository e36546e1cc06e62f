#!/bin/bash
# A K1 timing variant: tokcount_sl.hip compiled with extra defines and linked with the tree's
# other objects into lib/libtfidf_hip_<name>.so (selected by TFIDF_LIB=<name>).
#   bash scripts/k1_variant.sh <name> "<defines>" [source]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/parallel-systems-mpi-tfidf_amd
N=$1; D=$2; SRC=${3:-$P/csrc/tokcount_sl.hip}
mkdir -p $P/build/v_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I/opt/rocm/include -I$P/csrc $D -c $SRC -o $P/build/v_$N/tokcount_sl.o
O=""
for f in prims tokcount tokcount_vs finalize emit engine group ingest host_io; do O="$O $P/build/$f.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $P/lib/libtfidf_hip_$N.so $O $P/build/v_$N/tokcount_sl.o -L/opt/rocm/lib -lrccl -lm -Wl,-rpath,/opt/rocm/lib
echo "lib/libtfidf_hip_$N.so"
