#!/bin/bash
# MFMA tall F16 GEMV (lm_head, several columns): parity, then batched decode A/B
set -eo pipefail
OUT=gpurun_out/${1:-s2j}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_mul_mat_gpu.py tests/test_gpt2.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tall or batched or f16 or gpt2" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u tools/batched_tune.py f16_m8=1 f16_m8=0 f16_m8=1 f16_m8=0 > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
