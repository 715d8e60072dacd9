#!/bin/bash
# 8-wave LDS-staged planes kernel: parity + timing + stamps
set -eo pipefail
OUT=gpurun_out/${1:-r05n}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_gpu.py -k "planes or split_k or bit_equal" > "$OUT/pytest_planes.txt" 2>&1
tail -2 "$OUT/pytest_planes.txt"
PF_TYPES=q4_K PF_PLANES=1,0 PF_R=16 PF_SINGLE=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 > "$OUT/prefill_planes.txt" 2>&1
cat "$OUT/prefill_planes.txt"
timeout -k 10 120 python3 tools/mmqr_stamps.py 512 16 > "$OUT/mmqr_stamps.txt" 2>&1
head -8 "$OUT/mmqr_stamps.txt"
