#!/bin/bash
# k_mmq0x NR=2 + GEMV group balancing / Q4_0 pairs
set -eo pipefail
TAG=${1:-r03l}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export PF_TYPES=q4_0,q8_0 PF_R=32 MMQ_VARIANTS=0,$(( (1<<24) | 128 )),65664
timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 128 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf.txt"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu 2>&1 | grep --line-buffered -v amdgpu.ids > "$OUT/bench.json"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], json.dumps(d.get('sweep', {}))[:1500])"
