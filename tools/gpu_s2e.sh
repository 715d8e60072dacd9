#!/bin/bash
# register-quantizing norm prologue: parity (quantized GPT-2 / LLaMA block bit-identity, GEMV), then the A/B
set -eo pipefail
OUT=gpurun_out/${1:-s2e}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpt2.py tests/test_llama_block_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u tools/gpt2q_tune.py q4_k 3 mmv_pro4=1 mmv_pro4=0 > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
