#!/bin/bash
# k_mmqp weight ring (RING 4 vs 2, bit 2^19) and F16 k_mmf16p (vs k_mmq3, bit 2^18): prefill parity + timing at B = 128 / 64 / 32 (32 rotated weights)
set -eo pipefail
TAG=${1:-r03w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export PF_TYPES=q4_K,q5_K,f16 PF_R=32 MMQ_VARIANTS=0,524288,262144
timeout -k 10 300 python3 -u tools/prefill_bench.py 128 64 32 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
