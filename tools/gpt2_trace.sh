#!/bin/bash
# rocprofv3 kernel trace of GPT-2 decode (graph plans) -> per-kernel averages over the last 8 tokens
#   tools/gpt2_trace.sh <out tag> <kernels per token>   (env passes through, e.g. GGML_MI355X_FUSE_MASK)
set -eo pipefail
OUT=gpurun_out/${1:-gp}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv -- python3 tools/gpt2_prof.py 32 > "$OUT/log" 2>&1
grep -E "tok/s|per token" "$OUT/log"
python3 tools/trace_summary.py "$OUT/prof" ${2:-62} 8 | tee "$OUT/summary.txt"
