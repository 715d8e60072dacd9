#!/bin/bash
# Scratch A/B of the long-prompt kernels (round 4): mmq_long 1 k_mmqw, 2 k_mmqr, 3 k_mmqs
set -eo pipefail
OUT=gpurun_out/${1:-r04c}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K,q5_K PF_LONG=${PF_LONG:-1,3} MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py ${PF_B:-512 256} 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_long.txt
