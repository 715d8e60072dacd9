#!/bin/bash
# Q8_0 aligned copy: parity, then A/B against the canonical layout
set -eo pipefail
OUT=gpurun_out/${1:-s2i}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_q40_repack_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "q40 or q8_0 or q4_0" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/q40r_ab.py 3 q8_0 > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
