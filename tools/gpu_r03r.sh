#!/bin/bash
# warp-specialized k_mmqw vs k_mmqx
set -eo pipefail
TAG=${1:-r03r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export PF_TYPES=q4_K PF_R=32 MMQ_VARIANTS=0,$(( (1<<28) | 128 | 131072 ))
timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
