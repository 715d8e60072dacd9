#!/bin/bash
# prefill GEMM: parity tests (golden, config 5 shards) + timing
set -eo pipefail
OUT=gpurun_out/${1:-pf}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PF_TYPES=q4_K,q5_K timeout -k 10 200 python -u tools/prefill_bench.py 512 256 128 64 16 2>&1 | grep -v amdgpu.ids
