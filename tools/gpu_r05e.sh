#!/bin/bash
# 16-lane Q8_K prologue: parity tests, lone GEMV timings, stamps with shader clock
set -eo pipefail
OUT=gpurun_out/${1:-r05e}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
timeout -k 10 200 python3 -u tools/lone_gemv.py q4_K:4096:4096:1 q4_K:4096:11008:1 q5_K:4096:11008:1 q4_K:768:2304:1 q4_K:3072:768:1 f16:768:2304:1 > "$OUT/lone.txt" 2>&1
cat "$OUT/lone.txt"
timeout -k 10 200 python3 -u tools/stamps.py lone q4_K:4096:4096:1 q4_K:768:2304:1 f16:768:2304:1 > "$OUT/stamps_lone.txt" 2>&1
grep -A3 "==" "$OUT/stamps_lone.txt"
timeout -k 10 200 python3 -u tools/stamps.py gpt2 f16 8 > "$OUT/stamps_f16.txt" 2>&1
head -8 "$OUT/stamps_f16.txt"; tail -3 "$OUT/stamps_f16.txt"
timeout -k 10 200 python3 -u tools/stamps.py gpt2 q4_k 8 > "$OUT/stamps_q4k.txt" 2>&1
head -6 "$OUT/stamps_q4k.txt"; tail -3 "$OUT/stamps_q4k.txt"
timeout -k 10 200 python3 -u bench.py --no-cpu --no-sweep --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['gpt2']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_batched']['ms_per_step'])"
