#!/bin/bash
# Short-prompt Q4_K prefill diagnosis: kernel variants at B = 64 / 32 (32 rotated weights, grouped
# and one per graph) and k_mmqp's counters at B = 32 grouped (is it memory-throughput bound?)
set -eo pipefail
TAG=${1:-r03v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K PF_R=32
MMQ_VARIANTS=0,2048,65664,134217728,268435584 timeout -k 10 300 python3 -u tools/prefill_bench.py 64 32 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
export PF_SINGLE=0 MMQ_VARIANTS=0
timeout -k 10 400 python3 -u tools/pmc_kernel.py "$OUT/pmc" k_mmqp \
  'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY;TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE;TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum' \
  -- python3 tools/prefill_bench.py 32 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pmc.txt"
