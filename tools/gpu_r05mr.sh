#!/bin/bash
# multi-row tall GEMV: parity + decode bench + lm_head stamps
set -eo pipefail
OUT=gpurun_out/${1:-r05mr}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mul_mat_gpu.py -k "tall_short or quantized_decode" > "$OUT/pytest_mr.txt" 2>&1
tail -2 "$OUT/pytest_mr.txt"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_graphs_gpu.py > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
timeout -k 10 100 python3 tools/stamps.py lone q4_K:768:50257:1 > "$OUT/lone_lmhead.txt" 2>&1
tail -3 "$OUT/lone_lmhead.txt"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-sweep --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['gpt2']['ms_per_decode_token'], d['gpt2']['mmv_order_1']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_q4_k']['tree_order']['ms_per_decode_token'], d['gpt2_batched']['ms_per_step'])"
