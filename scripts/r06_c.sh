#!/bin/bash
# Round 6 call c: kernel traces of the two-pass K1 (default build and the 4-waves-per-SIMD K1a
# build), then an A/B of both against the fused default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TFIDF_K1=2p bash scripts/kstats.sh 2p --config c2 --no-emit --no-probe || { echo "kstats 2p failed"; exit 1; }
TFIDF_K1=2p TFIDF_LIB=ta4 bash scripts/kstats.sh 2p_ta4 --config c2 --no-emit --no-probe || { echo "kstats ta4 failed"; exit 1; }
VARIANTS="${VARIANTS:-base env:TFIDF_K1=2p env:TFIDF_K1=2p,TFIDF_LIB=ta4}" ROUNDS=${ROUNDS:-2} CFG=${CFG:-c2} bash scripts/r05_c.sh
