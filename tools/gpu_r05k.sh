#!/bin/bash
# round 5: repacked-planes prefill (k_mmqr) parity + timing, masked attention fusion, multi-column tall GEMV
set -eo pipefail
OUT=gpurun_out/${1:-r05k}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_gpu.py -k "planes" > "$OUT/pytest_planes.txt" 2>&1
tail -2 "$OUT/pytest_planes.txt"
PF_TYPES=q4_K,q5_K PF_PLANES=1,0 PF_R=16 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 136 > "$OUT/prefill_planes.txt" 2>&1
cat "$OUT/prefill_planes.txt"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_gpu.py tests/test_gpt2.py tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-sweep --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['gpt2']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_batched'])"
