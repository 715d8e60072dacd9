#!/bin/bash
# F16 short-prompt kernels under rocprof: per-kernel durations (k_mmf16p vs k_mmq3, convert) and
# k_mmf16p counters at B = 64
set -eo pipefail
TAG=${1:-r03z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=f16 PF_R=8 PF_SINGLE=0
MMQ_VARIANTS=0,262144 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 tools/prefill_bench.py 64 16 > "$OUT/prof.txt" 2>&1
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-8 "$OUT/kernel_stats.csv" | head -12
MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/pmc_kernel.py "$OUT/pmc" k_mmf16p \
  'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY;FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum' \
  -- python3 tools/prefill_bench.py 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc.txt"
