#!/bin/bash
# Round 6 call i: K5 emission A/B on c2 and c5: base (idf of 8 positions per lane gathered
# before their stores, 8 records per lane prefetched), em8 (the same with 4 prefetched),
# k5r5 (4 positions per lane per batch, round 5's batching).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
VARIANTS="${VARIANTS:-base em8 k5r5}" ROUNDS=${ROUNDS:-3} CFG=c2 bash scripts/r05_c.sh || exit 1
VARIANTS="${VARIANTS:-base em8 k5r5}" ROUNDS=1 CFG=c5 bash scripts/r05_c.sh || exit 1
