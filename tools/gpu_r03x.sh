#!/bin/bash
# F16 short-prompt k_mmf16p (vs k_mmq3: variant bit 2^18) and GPT-2 logits written by the lm_head
# GEMV into the pinned staging: parity tests + timing
set -eo pipefail
TAG=${1:-r03x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_mul_mat_gpu.py tests/test_gpt2.py tests/test_graphs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python3 -u tools/gpt2_prof.py 128 2>&1 | grep -v amdgpu.ids | tee "$OUT/gpt2.txt"
GPT2_QTYPE=q4_k timeout -k 10 120 python3 -u tools/gpt2_prof.py 128 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/gpt2.txt"
export PF_TYPES=f16 PF_R=16 MMQ_VARIANTS=0,262144
timeout -k 10 240 python3 -u tools/prefill_bench.py 128 64 32 16 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
