#!/bin/bash
# F16 decode checks: fast-mode parity tests + chain probe + GPT-2 decode timing
set -eo pipefail
OUT=gpurun_out/${1:-f16}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_mul_mat_gpu.py tests/test_gpt2.py -m gpu -x -v --timeout 120 --timeout-method thread -k "f16 or gpt2 or float or matches_reference" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python -u tools/chain_probe.py 50 > "$OUT/chain.log" 2>&1
cat "$OUT/chain.log"
timeout -k 10 120 python -u tools/gpt2_prof.py 128 > "$OUT/gpt2_prof.log" 2>&1
cat "$OUT/gpt2_prof.log"
