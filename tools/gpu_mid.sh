#!/bin/bash
# mid-batch prefill (k_mmqd, B <= 128): parity tests + timing of the variants in MMQ_VARIANTS
set -eo pipefail
OUT=gpurun_out/${1:-mid}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
MMQ_VARIANTS=${MMQ_VARIANTS:-0,256} PF_TYPES=${PF_TYPES:-q4_K,q5_K} timeout -k 10 200 python -u tools/prefill_bench.py ${BS:-128 64 32 16} 2>&1 | grep -v amdgpu.ids
