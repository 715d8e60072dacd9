#!/bin/bash
# load-order fixes in the decode GEMVs: parity tests + quick bench
set -eo pipefail
OUT=gpurun_out/${1:-r05t}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py tests/test_llama_block_gpu.py > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-sweep --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['gpt2']['ms_per_decode_token'], d['gpt2']['mmv_order_1']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_q4_k']['tree_order']['ms_per_decode_token'], d['gpt2_batched']['ms_per_step'])"
