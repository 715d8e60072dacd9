#!/bin/bash
# Q4_0 repacked decode GEMV: parity tests, then the A/B against the canonical layout
set -eo pipefail
OUT=gpurun_out/${1:-q40r}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_q40_repack_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "q40 or q4_0" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u tools/q40r_ab.py 3 > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
# k_mmqt (128 x 64 tiles, K split over wave pairs) against k_mmqp at short-prompt widths
PF_TYPES=q4_K PF_R=32 MMQ_VARIANTS=0,131200 PF_LONG=0 timeout -k 10 300 python -u tools/prefill_bench.py 64 128 32 > $OUT/pf_mmqt_short.txt 2>&1
cat $OUT/pf_mmqt_short.txt
