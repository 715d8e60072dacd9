#!/bin/bash
# round-3: prefill timing without the profiler (grouped and one per graph), then kernel durations
set -eo pipefail
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_TYPES=q4_K PF_R=32 timeout -k 10 200 python3 -u tools/prefill_bench.py 512 128 64 32 16 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
PF_TYPES=q4_K PF_R=32 PF_SINGLE=0 MMQ_VARIANTS=0,2048 timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 512 64 16 > "$OUT/pf_prof.txt" 2> "$OUT/pf_prof.err"
grep -v amdgpu.ids "$OUT/pf_prof.txt"
find "$OUT/pf" -name '*kernel_trace.csv' -exec cp {} "$OUT/pf_kernel_trace.csv" \;
python3 tools/ktrace.py "$OUT/pf_kernel_trace.csv"
