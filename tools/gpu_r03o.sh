#!/bin/bash
# quantized GPT-2 default-order error per type; GPT-2 f16 decode trace
set -eo pipefail
TAG=${1:-r03o}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpt2.py -m gpu -x -v -s -k "default_order" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
grep -E "default order max|passed|failed" "$OUT/pytest.log"
bash tools/gpt2_trace.sh $TAG/f16 50
