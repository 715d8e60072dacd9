#!/bin/bash
# k_mmf16p with 8 waves per tile (variant bit 2^20) vs 4 (default) vs k_mmq3 (2^18): F16 parity under
# the 8-wave variant + timing
set -eo pipefail
TAG=${1:-r03aa}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GGML_MI355X_MMQ_VARIANT=1048576 timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "f16 or shapes or broadcast" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export PF_TYPES=f16 PF_R=16
MMQ_VARIANTS=0,1048576 timeout -k 10 250 python3 -u tools/prefill_bench.py 128 64 32 16 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
