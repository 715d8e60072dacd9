#!/bin/bash
# Scratch A/B + targeted GPU tests of the work in progress (round 4)
set -eo pipefail
OUT=gpurun_out/${1:-r04b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K,q5_K PF_LONG=1,2 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_long.txt
timeout -k 10 600 python -u -m pytest tests/test_gpt2.py -x -v --timeout 300 --timeout-method thread -m gpu -k "batched or default_order" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "PASS|FAIL|max rel|identical" $OUT/pytest.log | tail -30
