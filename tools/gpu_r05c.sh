#!/bin/bash
# activation-first (xfirst) A/B: lone GEMVs and GPT-2 decode, stamps + timings; GEMV/GPT-2 parity tests
set -eo pipefail
OUT=gpurun_out/${1:-r05c}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CASES="q4_K:4096:4096:1 q4_K:768:2304:1 q4_K:3072:768:1 q4_0:4096:4096:1 q8_0:4096:11008:1 q5_K:4096:11008:1 f16:768:2304:1"
for XF in 1 0; do
  GGML_MI355X_XFIRST=$XF timeout -k 10 200 python3 -u tools/lone_gemv.py $CASES > "$OUT/lone_xf$XF.txt" 2>&1
  cat "$OUT/lone_xf$XF.txt"
done
GGML_MI355X_XFIRST=1 timeout -k 10 200 python3 -u tools/stamps.py lone q4_K:4096:4096:1 q4_K:768:2304:1 f16:768:2304:1 > "$OUT/stamps_lone.txt" 2>&1
cat "$OUT/stamps_lone.txt"
for XF in 1 0; do
  GGML_MI355X_XFIRST=$XF timeout -k 10 200 python3 -u tools/stamps.py gpt2 f16 8 > "$OUT/gpt2_f16_xf$XF.txt" 2>&1
  tail -3 "$OUT/gpt2_f16_xf$XF.txt"
  GGML_MI355X_XFIRST=$XF timeout -k 10 200 python3 -u tools/stamps.py gpt2 q4_k 8 > "$OUT/gpt2_q4k_xf$XF.txt" 2>&1
  tail -3 "$OUT/gpt2_q4k_xf$XF.txt"
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_gpt2.py tests/test_prefill_gpu.py tests/test_llama_block_gpu.py tests/test_bench_gpu.py -k "not full_size" > "$OUT/pytest.txt" 2>&1
tail -5 "$OUT/pytest.txt"
