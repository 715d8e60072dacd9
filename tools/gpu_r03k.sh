#!/bin/bash
# Q4_0 GEMV item formats (single blocks vs pairs) + k_mmq0x counters
set -eo pipefail
TAG=${1:-r03k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GGML_MI355X_MMV_VARIANT=12 timeout -k 10 200 python -u -m pytest tests/test_mul_mat_gpu.py -m gpu -x -q -k "q4_0" --timeout 120 --timeout-method thread > "$OUT/pytest_pairs.log" 2>&1 || { tail -30 "$OUT/pytest_pairs.log"; exit 1; }
tail -1 "$OUT/pytest_pairs.log"
timeout -k 10 200 python3 -u tools/mmv_tune.py --type q4_0 --variants 11:0,12:0,22:0,32:0,21:0 --rounds 7 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/tune_q4_0.txt"
timeout -k 10 200 python3 -u tools/mmv_tune.py --type q4_0 --N 11008 --variants 11:0,12:0,22:0 --rounds 5 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/tune_q4_0_11008.txt"
export PF_TYPES=q4_0 PF_SINGLE=0 MMQ_VARIANTS=0
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM"
C2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
timeout -k 10 250 python3 tools/pmc_kernel.py "$OUT/pmc" mmq0x "$C1;$C2" -- python3 tools/prefill_bench.py 512 > "$OUT/pmc.txt" 2>&1 || true
cat "$OUT/pmc.txt"
