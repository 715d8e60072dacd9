#!/bin/bash
# Round 4: parity after the GEMV default change, then k_mmqt SPLIT 2 (mmq_long 7) A/B
set -eo pipefail
OUT=gpurun_out/${1:-r04t}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_mul_mat_gpu.py tests/test_prefill_gpu.py tests/test_gpt2.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K PF_LONG=0,7,0,7 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf.txt
