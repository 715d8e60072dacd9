#!/bin/bash
# Q4_K (bit-identical default) and f16 GPT-2 decode kernel traces
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GPT2_QTYPE=q4_k bash tools/gpt2_trace.sh ${1:-s2g}_q4k 62
bash tools/gpt2_trace.sh ${1:-s2g}_f16 50
