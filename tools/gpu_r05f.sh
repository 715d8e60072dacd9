#!/bin/bash
set -eo pipefail
OUT=gpurun_out/${1:-r05f}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_gpt2.py -k "quantized or mul_mat or epilogue or fused" > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
timeout -k 10 200 python3 -u tools/stamps.py gpt2 q4_k 8 > "$OUT/stamps_q4k.txt" 2>&1
head -12 "$OUT/stamps_q4k.txt"; tail -3 "$OUT/stamps_q4k.txt"
timeout -k 10 200 python3 -u tools/gpt2_prof.py 64 > "$OUT/gpt2.txt" 2>&1; grep tok/s "$OUT/gpt2.txt"
GPT2_QTYPE=q4_k timeout -k 10 200 python3 -u tools/gpt2_prof.py 64 > "$OUT/gpt2q.txt" 2>&1; grep -E "tok/s|per token" "$OUT/gpt2q.txt"
