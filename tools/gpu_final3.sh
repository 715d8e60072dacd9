#!/bin/bash
# Round-3 final pass: every GPU test, smoke(), the bench line, the headline alone under rocprof
# (dominant kernel duration vs the bench's roofline) and the F16 short-prompt timings
set -eo pipefail
TAG=${1:-final3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -5 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'frac', d['roofline']['frac'], 'gpt2', d['gpt2']['decode_tokens_per_s'], 'q4k', d['gpt2_q4_k']['decode_tokens_per_s'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_head" -o run --output-format csv -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu --no-gpt2 --no-sweep > "$OUT/head_bench.json" 2> "$OUT/head_prof.err"
find "$OUT/prof_head" -name '*kernel_stats.csv' -exec cp {} "$OUT/head_kernel_stats.csv" \;
head -3 "$OUT/head_kernel_stats.csv" | cut -c1-200
export PF_TYPES=f16 PF_R=16
MMQ_VARIANTS=0,262144 timeout -k 10 200 python3 -u tools/prefill_bench.py 128 64 32 16 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/pf_f16.txt"
