#!/bin/bash
# Round 6 call d: two-pass K1 with super-round counting: A/B, then K1a/K1b counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
VARIANTS="${VARIANTS:-base env:TFIDF_K1=2p env:TFIDF_K1=2p,TFIDF_LIB=ta4}" ROUNDS=${ROUNDS:-2} CFG=${CFG:-c2} bash scripts/r05_c.sh || exit 1
export TFIDF_K1=2p TFIDF_LIB=${PLIB:-ta4}
KREGEX=k_tok_ PASSES=2 bash scripts/prof_k1.sh 2p > /dev/null 2>&1
for k in k_tok_resolve k_tok_count; do echo "## $k"; python3 scripts/pmc_summary.py gpurun_out/prof_2p $k; done
