#!/bin/bash
# RCCL row leg with Q8_K broadcast; default bench run (prefill sweep rotated over 32 weights)
set -eo pipefail
TAG=${1:-r03n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 python3 -u bench.py 2>&1 | grep --line-buffered -v amdgpu.ids > "$OUT/bench.json"
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print(d['value'], d['ms_per_step'], json.dumps(d['cpu_baseline'])[:300])
for k,v in d['sweep'].items(): print(k, {kk:vv for kk,vv in v.items() if kk not in ('roofline','note')})
print(json.dumps(d.get('gpt2'))[:300]); print(json.dumps(d.get('gpt2_q4_k'))[:300])
"
