#!/bin/bash
# short prompts as 8-column tree-order GEMV chunks (tree_prefill_cols) vs the MFMA GEMMs
set -eo pipefail
OUT=gpurun_out/${1:-s2f}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for T in 0 64; do
  for ty in q4_K q4_0; do
    GGML_MI355X_TREE_PREFILL_COLS=$T PF_TYPES=$ty PF_R=32 MMQ_VARIANTS=0 timeout -k 10 200 python -u tools/prefill_bench.py 9 16 24 32 48 > $OUT/pf_${ty}_T$T.txt 2>&1
    grep -E "q4_" $OUT/pf_${ty}_T$T.txt | sed "s/^/T=$T /"
  done
done
