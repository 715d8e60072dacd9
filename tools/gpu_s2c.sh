#!/bin/bash
# k_mmqt short-prompt threshold: always-on vs off at small groups
set -eo pipefail
OUT=gpurun_out/${1:-s2c}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in 1 2 3 4 6; do
  for T in 1 0; do
    GGML_MI355X_MMQT_SHORT=$T PF_TYPES=q4_K PF_R=$R PF_SINGLE=0 MMQ_VARIANTS=0 timeout -k 10 200 python -u tools/prefill_bench.py 48 64 96 128 > $OUT/pf_R${R}_T$T.txt 2>&1
    grep q4_K $OUT/pf_R${R}_T$T.txt | sed "s/^/T=$T /"
  done
done
