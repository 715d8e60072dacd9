#!/bin/bash
# round-3: prefill parity (new layout / fold / k_mmqp), then kernel timing (k_mmqp vs k_mmqd1)
set -eo pipefail
TAG=${1:-r03d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py tests/test_split_gpu.py tests/test_graphs_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
PF_TYPES=q4_K,q5_K PF_R=32 MMQ_VARIANTS=0,2048 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 512 128 64 32 > "$OUT/pf.txt" 2> "$OUT/pf.err"
grep -v amdgpu.ids "$OUT/pf.txt"
find "$OUT/pf" -name '*kernel_trace.csv' -exec cp {} "$OUT/pf_kernel_trace.csv" \;
python3 tools/ktrace.py "$OUT/pf_kernel_trace.csv"
