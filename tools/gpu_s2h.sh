#!/bin/bash
# staggered k_mmqt (mmq_long 5) vs plain (2): bit-equality, then the prefill A/B
set -eo pipefail
OUT=gpurun_out/${1:-s2h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_prefill_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for p in 1 2; do
  PF_TYPES=q4_K PF_R=16 PF_SINGLE=0 MMQ_VARIANTS=0 PF_LONG=2,5 timeout -k 10 300 python -u tools/prefill_bench.py 512 256 128 64 > $OUT/ab_$p.txt 2>&1
  grep q4_K $OUT/ab_$p.txt
done
