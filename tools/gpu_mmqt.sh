#!/bin/bash
# Round 4: the split-K long-prompt kernel (k_mmqt, mmq_long 2 / 6) -- Q4_K / Q5_K B=512 / 256 timing
# against the default, prefill parity (the canonical order changed for every Q4_K / Q5_K kernel),
# then one PMC pass set of k_mmqt
set -eo pipefail
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=0 PF_R=16 PF_TYPES=${PF_TYPES:-q4_K,q5_K} PF_LONG=${PF_LONG:-0,2,6} MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_long.txt
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_prefill.log 2>&1 && tail -1 $OUT/pytest_prefill.log || { grep -E "FAILED|^E " $OUT/pytest_prefill.log | head -20; tail -1 $OUT/pytest_prefill.log; }
if [ -z "$NO_PMC" ]; then
export PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K MMQ_VARIANTS=0
PF_LONG=2 timeout -k 10 300 python3 -u tools/pmc_kernel.py "$OUT/pmc_l2" k_mmq \
  'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY;GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY' \
  -- python3 tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc_l2.txt"
fi
