#!/bin/bash
# phase stamps of the Q4_K (reference order) and f16 GPT-2 decode token (diagnostic build)
set -eo pipefail
OUT=gpurun_out/${1:-s2m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/stamps.py gpt2 q4_k 8 > $OUT/q4k_stamps.txt 2>&1
cat $OUT/q4k_stamps.txt | head -30
timeout -k 10 300 python -u tools/stamps.py gpt2 f16 8 > $OUT/f16_stamps.txt 2>&1
head -12 $OUT/f16_stamps.txt
