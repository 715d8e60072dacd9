#!/bin/bash
# PMC counters of the grouped k_mmqp (B=64) and k_mmqx (B=512) launches
set -eo pipefail
TAG=${1:-r03g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K PF_R=32 PF_SINGLE=0
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
C3="TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
for B in 64 512; do
  timeout -k 10 250 python3 tools/pmc_kernel.py "$OUT/pmc_b$B" k_mmq "$C1;$C2" -- python3 tools/prefill_bench.py $B > "$OUT/pmc_b$B.txt" 2>&1 || { cat "$OUT/pmc_b$B.txt" | tail; exit 1; }
  cat "$OUT/pmc_b$B.txt"
done
timeout -k 10 120 python3 tools/pmc_kernel.py "$OUT/pmc_ta" k_mmqp "$C3" -- python3 tools/prefill_bench.py 64 > "$OUT/pmc_ta.txt" 2>&1 || true
cat "$OUT/pmc_ta.txt"
