#!/bin/bash
# Round 6 call a: K1 phase stamps of the current tree (c2), then timing ablations
# (base / ablw = no record writes / l2c = no record writes + every step's corpus from L2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06a
mkdir -p $OUT
cd $R
TFIDF_LIB=stamps TFIDF_STAMPS=1 timeout -k 10 240 python3 -u scripts/k1_stamps.py c2 > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -5 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
VARIANTS="${VARIANTS:-base ablw l2c}" ROUNDS=${ROUNDS:-2} bash scripts/r05_c.sh
