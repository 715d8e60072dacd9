#!/bin/bash
# k_mmqp (8 waves, SWAR factors) parity + timing, single and grouped
set -eo pipefail
TAG=${1:-r03h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"

export PF_TYPES=q4_K PF_R=32 MMQ_VARIANTS=0,$((1<<27)),2048
timeout -k 10 300 python3 -u tools/prefill_bench.py 64 32 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
export PF_TYPES=q4_K PF_SINGLE=0 MMQ_VARIANTS=0,$((1<<27))
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM"
timeout -k 10 250 python3 tools/pmc_kernel.py "$OUT/pmc" mmqp "$C1" -- python3 tools/prefill_bench.py 64 > "$OUT/pmc.txt" 2>&1 || true
cat "$OUT/pmc.txt"
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/pf" -o run --output-format csv -- python3 tools/prefill_bench.py 64 > "$OUT/pf_prof.txt" 2> "$OUT/pf_prof.err"
find "$OUT/pf" -name '*kernel_trace.csv' -exec cp {} "$OUT/pf_kernel_trace.csv" \;
python3 tools/ktrace.py "$OUT/pf_kernel_trace.csv"
