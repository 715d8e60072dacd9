#!/bin/bash
# Evidence pass (round 4):
#  1. long-prompt kernels A/B (k_mmqw vs k_mmqr), bit-equality against the first
#  2. PMC HBM traffic of HEAD's k_mmv_stream (tools/pmc_traffic.py, separate FETCH/WRITE passes)
#  3. rocprof kernel durations of one Q4_K 4096^2 GEMV per graph (and grouped), B=1
#  4. PMC pass of the default B=512 prefill kernel (MFMA busy, VALU/MFMA, LDS bank conflicts)
set -eo pipefail
TAG=${1:-r04a}
KPMC=${2:-k_mmqw}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=1 PF_TYPES=q4_K,q5_K PF_LONG=1,2 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 \
  | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf_long.txt"
timeout -k 10 300 python3 -u tools/pmc_traffic.py --tag "$TAG" > "$OUT/pmc_traffic.log" 2>&1
grep -A3 k_mmv_stream "$OUT/pmc_traffic.log" | head -8 || true
export PF_TYPES=q4_K PF_R=32
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_single" -o run --output-format csv -- \
  python3 tools/prefill_bench.py 1 > "$OUT/single.txt" 2>&1
find "$OUT/prof_single" -name '*kernel_stats.csv' -exec cp {} "$OUT/single_kernel_stats.csv" \;
grep -v amdgpu.ids "$OUT/single.txt" | tail -2
cut -c1-160 "$OUT/single_kernel_stats.csv" | head -6
export PF_SINGLE=0
timeout -k 10 400 python3 -u tools/pmc_kernel.py "$OUT/pmc_long" "$KPMC" \
  'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY;GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES;FETCH_SIZE' \
  -- python3 tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc_long.txt"
