#!/bin/bash
# Round 4 A/B: k_mmqt DMAs through buffer descriptors (mmq_long 5) vs per-lane addresses (0), with
# bit-equality; then the config-2/3 GEMV sweep
set -eo pipefail
OUT=gpurun_out/${1:-r04p}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K PF_LONG=0,5,6,0,5,6 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf.txt
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "split_k or bit_equal" > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
bash tools/gpu_gemv_sweep.sh ${1:-r04p}
