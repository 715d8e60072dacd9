#!/bin/bash
# F16 short-prompt k_mmf16p (coalesced loads, LDS-staged weights): parity, timing vs k_mmq3
# (variant bit 2^18) and per-kernel durations under rocprof
set -eo pipefail
TAG=${1:-r03z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "f16 or shapes or broadcast" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export PF_TYPES=f16 PF_R=16
MMQ_VARIANTS=0,262144 timeout -k 10 200 python3 -u tools/prefill_bench.py 128 64 32 16 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
export PF_R=8 PF_SINGLE=0
MMQ_VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 tools/prefill_bench.py 64 16 > "$OUT/prof.txt" 2>&1
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | cut -c1-150
