#!/bin/bash
# Final pass of a round: the whole -m gpu suite, smoke(), and a rocprof kernel trace of the
# headline alone (no sweep / GPT-2 / CPU legs) so the dominant kernel's average duration can be
# compared with bench.py's roofline directly.
set -eo pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -6 "$OUT/smoke.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_head" -o run --output-format csv -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu --no-gpt2 --no-sweep > "$OUT/head_bench.json" 2> "$OUT/head_prof.err"
find "$OUT/prof_head" -name '*kernel_stats.csv' -exec cp {} "$OUT/head_kernel_stats.csv" \;
head -4 "$OUT/head_kernel_stats.csv" | cut -c1-220
python3 -c "import json; d=json.load(open('$OUT/head_bench.json')); print('roofline achieved', d['roofline']['achieved'], 'event_ms', d['roofline']['event_ms_per_step'])"
