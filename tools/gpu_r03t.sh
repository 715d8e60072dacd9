#!/bin/bash
# k_mmqw stage timing stamps (results invalid), B=512 and 256
set -eo pipefail
TAG=${1:-r03t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STAMP_VARIANT=$((1<<29)) timeout -k 10 120 python3 -u tools/mmqx_stamps.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/stamps512.txt"
STAMP_VARIANT=0 timeout -k 10 120 python3 -u tools/mmqx_stamps.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/stamps512_mmqx.txt"
