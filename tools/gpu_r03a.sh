#!/bin/bash
# round-3 check: full GPU parity suite, then the bench line (GEMV + sweep + GPT-2)
set -eo pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('sweep',{}))); g=d.get('gpt2',{}); print(g.get('decode_tokens_per_s'), g.get('graphs')); print(d.get('gpt2_q4_k',{}).get('decode_tokens_per_s'))"
