#!/bin/bash
# PMC passes of the long-prompt kernels at B=512 (Q4_K): one rocprofv3 pass per counter group
set -eo pipefail
OUT=gpurun_out/${1:-r04d}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K MMQ_VARIANTS=0
for L in ${PF_LONGS:-4 3}; do
  PF_LONG=$L timeout -k 10 300 python3 -u tools/pmc_kernel.py "$OUT/pmc_l$L" k_mmq \
    'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY;GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY;SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS' \
    -- python3 tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc_l$L.txt"
done
