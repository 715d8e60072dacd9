#!/bin/bash
# round-3: prefill + graph tests, launch floor probe, grouped vs single prefill timing
set -eo pipefail
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py tests/test_graphs_gpu.py tests/test_gpt2.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 120 tools/kfloor > "$OUT/kfloor.txt" 2>&1
cat "$OUT/kfloor.txt"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/kf" -o run --output-format csv -- tools/kfloor > /dev/null 2>&1
find "$OUT/kf" -name '*kernel_stats.csv' -exec cp {} "$OUT/kfloor_kernel_stats.csv" \;
cut -d, -f1-7 "$OUT/kfloor_kernel_stats.csv"
# grouped (R mul_mats per graph, 16 per group) vs one mul_mat per graph
PF_TYPES=q4_K PF_R=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 512 64 16 > "$OUT/pf.txt" 2> "$OUT/pf.err"
grep -v amdgpu.ids "$OUT/pf.txt"
find "$OUT/pf" -name '*kernel_stats.csv' -exec cp {} "$OUT/pf_kernel_stats.csv" \;
cut -d, -f1-7 "$OUT/pf_kernel_stats.csv" | cut -c1-220
