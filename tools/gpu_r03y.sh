#!/bin/bash
# GPT-2 decode on one box: logits by in-graph CPY (default) vs a copy queued behind the graph
# (GPT2_LOGITS_COPY=1), each with plan-launch flush 1 (marker event) and 2 (hipStreamQuery)
set -eo pipefail
TAG=${1:-r03y}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for lc in 0 1; do
for f in 1 2; do
  echo "rep=$rep LOGITS_COPY=$lc PLAN_FLUSH=$f" | tee -a "$OUT/gpt2.txt"
  GPT2_LOGITS_COPY=$lc GGML_MI355X_PLAN_FLUSH=$f timeout -k 10 120 python3 -u tools/gpt2_prof.py 128 2>&1 | grep -v amdgpu.ids | grep -E "decode|per token" | tee -a "$OUT/gpt2.txt"
done
done
done
