#!/bin/bash
# One GPU-box pass: parity tests, the bench line, a rocprofv3 kernel-trace summary of the same
# bench, and the PMC traffic passes. Every GPU step has its own time limit and the steps are
# chained so that the first failure ends the call.
#   usage: gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG [skip-tests]
set -eo pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu --no-gpt2 --no-sweep > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
head -8 "$OUT/kernel_stats.csv" | cut -c1-200
timeout -k 10 300 python tools/pmc_traffic.py --tag "$TAG" > "$OUT/pmc.log" 2>&1
tail -5 "$OUT/pmc.log"
# GPT-2 decode kernel trace (per-token launch mix)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gpt2" -o run --output-format csv -- \
  python3 tools/gpt2_prof.py 64 > "$OUT/gpt2_prof.log" 2>&1
find "$OUT/prof_gpt2" -name '*kernel_stats.csv' -exec cp {} "$OUT/gpt2_kernel_stats.csv" \;
cat "$OUT/gpt2_prof.log" | tail -4
# GPT-2 per-kernel decode durations over the last tokens
bash tools/gpt2_trace.sh "$TAG/gpt2_trace" 51 | tail -12
# prefill GEMM counters (k_mmqt, the Q4_K default at B = 512): MFMA busy, VALU per MFMA, waits
timeout -k 10 300 python tools/pmc_kernel.py "$OUT/pmc_mmqt" k_mmqt "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" -- python3 tools/prefill_bench.py 512 > "$OUT/mmqt_pmc.txt" 2>&1
grep -E "MFMA|VALU" "$OUT/mmqt_pmc.txt" | head -6
