#!/bin/bash
# per-kernel durations of the batched prefill mul_mat (quantizer + GEMM) at several B
set -o pipefail
OUT=gpurun_out/${1:-pft}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 512 64 16; do
  PF_TYPES=q4_K timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/b$B" -o run --output-format csv -- python3 tools/prefill_bench.py $B > "$OUT/b$B.log" 2>&1 || exit 1
  grep "us/mul_mat" "$OUT/b$B.log"
  f=$(find "$OUT/b$B" -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | cut -c1-150
done
