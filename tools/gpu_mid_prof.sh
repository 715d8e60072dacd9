#!/bin/bash
# k_mmqd per-kernel durations (rocprofv3 kernel trace) over the MMQ_VARIANTS ablations
set -eo pipefail
OUT=gpurun_out/${1:-midprof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MMQ_VARIANTS=${MMQ_VARIANTS:-256} PF_TYPES=${PF_TYPES:-q4_K}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 tools/prefill_bench.py ${BS:-64} > "$OUT/bench.txt" 2> "$OUT/prof.err"
grep -v amdgpu.ids "$OUT/bench.txt"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -c1-160 "$OUT/kernel_stats.csv" | head -20
