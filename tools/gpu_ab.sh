#!/bin/bash
# Scratch A/B of work in progress (round 4): long-prompt kernels (mmq_long 1 k_mmqw, 3 k_mmqs,
# 4 k_mmqs rolled) and the F16 short-prompt GEMM with the conversion folded in (bit 2^17 = old path)
set -eo pipefail
OUT=gpurun_out/${1:-r04c}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=0 PF_R=16 PF_TYPES=${PF_TYPES:-q4_K} PF_LONG=${PF_LONG:-1,2,4} MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_long.txt
PF_SINGLE=1 PF_R=16 PF_TYPES=f16 MMQ_VARIANTS=0,131072 timeout -k 10 300 python3 -u tools/prefill_bench.py 64 32 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_f16.txt
timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "f16 or float" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
# single-GEMV graphs: the decode GEMV's grid target (0 = automatic, 1024 WGs here)
PF_SINGLE=1 PF_R=32 PF_TYPES=q4_K PF_MMV_BLOCKS=0,256,512 timeout -k 10 300 python3 -u tools/prefill_bench.py 1 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_single_blocks.txt
