#!/bin/bash
# spin-polled synchronize (sync_spin) A/B: GPT-2 f16 decode and batched decode
set -eo pipefail
OUT=gpurun_out/${1:-s2l}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/gpt2_tune.py sync_spin=0 sync_spin=1 sync_spin=0 sync_spin=1 > $OUT/gpt2_ab.txt 2>&1
cat $OUT/gpt2_ab.txt
timeout -k 10 300 python -u tools/batched_tune.py sync_spin=1 sync_spin=0 sync_spin=1 sync_spin=0 > $OUT/batched_ab.txt 2>&1
cat $OUT/batched_ab.txt
