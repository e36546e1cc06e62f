#!/bin/bash
# A timing variant: one source file compiled with extra defines and linked with the tree's
# other objects into lib/libtfidf_hip_<name>.so (selected by TFIDF_LIB=<name>).
#   bash scripts/k1_variant.sh <name> "<defines>" [source file, default csrc/tokcount_sl.hip]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/parallel-systems-mpi-tfidf_amd
N=$1; D=$2; SRC=${3:-$P/csrc/tokcount_sl.hip}
B=$(basename $SRC .hip)
mkdir -p $P/build/v_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I/opt/rocm/include -I$P/csrc $D -c $SRC -o $P/build/v_$N/$B.o
O=""
for f in prims tokcount tokcount_vs tokcount_sl finalize emit engine group ingest host_io; do
  if [ $f = $B ]; then O="$O $P/build/v_$N/$B.o"; else O="$O $P/build/$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $P/lib/libtfidf_hip_$N.so $O -L/opt/rocm/lib -lrccl -lm -Wl,-rpath,/opt/rocm/lib
echo "lib/libtfidf_hip_$N.so"
