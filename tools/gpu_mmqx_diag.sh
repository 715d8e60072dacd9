#!/bin/bash
# k_mmqx diagnostics: timing ablations + SQ / MFMA counters at B=512 and B=64
set -o pipefail
OUT=gpurun_out/${1:-mmqx}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K
for v in 0 256 512 768 1024 1792; do
  echo "variant $v" >> "$OUT/abl.txt"
  GGML_MI355X_MMQ_VARIANT=$v timeout -k 10 120 python -u tools/prefill_bench.py 512 64 2>&1 | grep -v amdgpu.ids >> "$OUT/abl.txt" || exit 1
done
cat "$OUT/abl.txt"
timeout -k 10 300 python tools/pmc_kernel.py "$OUT/pmc" k_mmqx "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE;SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT" -- python3 tools/prefill_bench.py 512 > "$OUT/pmc.txt" 2>&1
cat "$OUT/pmc.txt"
