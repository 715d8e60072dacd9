#!/bin/bash
# Round 4: k_mmqt with skewed halves (mmq_long 7) against k_mmqt (0) and k_mmqw (1), both builds
set -eo pipefail
OUT=gpurun_out/${1:-r04k}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for LIBV in main pk main; do
  if [ $LIBV = pk ]; then export GGML_MI355X_BACKEND_LIB=$GRAFT_REPO_ROOT/ggml-imax_amd/lib/pk/libggml_mi355x.so; else unset GGML_MI355X_BACKEND_LIB; fi
  echo "== $LIBV" | tee -a $OUT/pf.txt
  PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K PF_LONG=0,7,1 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee -a $OUT/pf.txt
done
unset GGML_MI355X_BACKEND_LIB
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "split_k or bit_equal" > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; }
export PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K MMQ_VARIANTS=0
PF_LONG=7 timeout -k 10 300 python3 -u tools/pmc_kernel.py "$OUT/pmc_s" k_mmq \
  'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY;GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY' \
  -- python3 tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc_s.txt"
