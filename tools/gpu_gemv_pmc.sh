#!/bin/bash
# Round 4: counters of the default GEMV kernel for Q4_0 4096^2 (config 2) beside Q4_K 4096^2 (the
# headline) and Q8_0 4096x11008: issue, VMEM / TA / TCP stalls (one rocprofv3 --pmc pass per group)
set -eo pipefail
OUT=gpurun_out/${1:-r04pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
G="SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE;TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE;TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum;TD_TD_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
for spec in "q4_0 4096 4096 36 32:0" "q4_K 4096 4096 32 31:0" "q8_0 4096 11008 8 11:0"; do
  set -- $spec
  echo "== $1 ${2}x${3} variant $5" | tee -a $OUT/gemv_pmc.txt
  timeout -k 10 400 python3 -u tools/pmc_kernel.py $OUT/p_$1 k_mmv_stream "$G" -- python3 tools/mmv_tune.py --variants $5 --rounds 2 --type $1 --K $2 --N $3 --rotate $4 2>&1 | tee -a $OUT/gemv_pmc.txt
done
