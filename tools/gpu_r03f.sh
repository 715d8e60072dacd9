#!/bin/bash
# k_mmqp ablations at B=64 (single and grouped), events then kernel trace
set -eo pipefail
TAG=${1:-r03f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "float_mul_mat or f16_src1" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
export PF_TYPES=q4_K PF_R=32 MMQ_VARIANTS=0,4096,8192,12288,16384,28672
timeout -k 10 200 python3 -u tools/prefill_bench.py 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 64 > "$OUT/pf_prof.txt" 2> "$OUT/pf_prof.err"
find "$OUT/pf" -name '*kernel_trace.csv' -exec cp {} "$OUT/pf_kernel_trace.csv" \;
python3 tools/ktrace.py "$OUT/pf_kernel_trace.csv"
