#!/bin/bash
# Round 4: quick parity of the fused canonical fold and the graph_compute rule
set -eo pipefail
OUT=gpurun_out/${1:-r04w}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_graphs_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K,q5_K MMQ_VARIANTS=0 PF_LONG=0,1 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf.txt
# one GEMV per graph: grid of 128 / 192 / 256 workgroups (0 = the automatic choice)
PF_SINGLE=1 PF_R=32 PF_TYPES=q4_K PF_MMV_BLOCKS=0,128,192,256 timeout -k 10 300 python3 -u tools/prefill_bench.py 1 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_single.txt
