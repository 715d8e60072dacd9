#!/bin/bash
# interleaved-slice Q8_K prologue: parity (norm-prologue GEMVs, GPT-2 / llama bit identity) + GPT-2 Q4_K decode A/B
set -eo pipefail
OUT=gpurun_out/${1:-s2n}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_gpt2.py tests/test_llama_block_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
timeout -k 10 300 python -u tools/gpt2q_tune.py q4_k 3 mmv_pro4=1 mmv_pro4=0 > $OUT/gpt2q_ab.txt 2>&1
cat $OUT/gpt2q_ab.txt
