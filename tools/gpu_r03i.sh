#!/bin/bash
# exact Q4_0 / Q8_0 prefill (k_mmq0p): parity + timing
set -eo pipefail
TAG=${1:-r03i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
export PF_TYPES=q4_0,q8_0 PF_R=32 MMQ_VARIANTS=0,16,65664
timeout -k 10 300 python3 -u tools/prefill_bench.py 512 128 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
export PF_SINGLE=0 PF_TYPES=q4_0
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 512 64 > "$OUT/pf_prof.txt" 2> "$OUT/pf_prof.err"
find "$OUT/pf" -name '*kernel_stats.csv' -exec cp {} "$OUT/pf_kernel_stats.csv" \;
cut -c1-160 "$OUT/pf_kernel_stats.csv" | head -12
