#!/bin/bash
set -eo pipefail
OUT=gpurun_out/${1:-r05j}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py -k "batched or f16 or float or logits or graph" > "$OUT/pytest.txt" 2>&1
tail -2 "$OUT/pytest.txt"
for B in 1 8; do timeout -k 10 100 python3 tools/stamps.py normgemv 768 2304 $B | head -4; done
timeout -k 10 300 python3 -u bench.py --no-cpu --no-sweep --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['gpt2']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_batched']['ms_per_step'])"
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 tools/batched_prof.py > $OUT/prof_log.txt 2>&1
python3 tools/trace_summary.py $OUT/prof 134 8 | head -14
