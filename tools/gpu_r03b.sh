#!/bin/bash
# round-3: GPU parity suite + bench, then k_mmqd1 access-pattern ablations under rocprof
set -eo pipefail
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('sweep',{}))); g=d.get('gpt2',{}); print(g.get('decode_tokens_per_s'), g.get('graphs'), g.get('host_us_per_token')); print(d.get('gpt2_q4_k',{}).get('decode_tokens_per_s'))"
# k_mmqd1 B=64: base, ABL 16 (repacked-weight addressing), 32 (activation [K/32] addressing), 48, 15 (all removed)
export PF_TYPES=q4_K PF_R=36 MMQ_VARIANTS=$(( 1<<21 )),$(( (1<<21) | (1<<23) )),$(( (1<<21) | (1<<24) )),$(( (1<<21) | (3<<23) )),$(( (1<<21) | (15<<12) ))
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/abl" -o run --output-format csv -- python3 tools/prefill_bench.py 64 > "$OUT/abl.txt" 2> "$OUT/abl.err"
grep -v amdgpu.ids "$OUT/abl.txt"
find "$OUT/abl" -name '*kernel_stats.csv' -exec cp {} "$OUT/abl_kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/abl_kernel_stats.csv" | cut -c1-170
unset MMQ_VARIANTS
PF_R=36 timeout -k 10 200 python -u tools/prefill_bench.py 512 64 32 16 2>&1 | grep -v amdgpu.ids
