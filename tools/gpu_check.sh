#!/bin/bash
# Round-end check: every GPU test, smoke(), the bench line and a kernel trace of the prefill sizes
set -eo pipefail
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.txt" 2>&1
cat "$OUT/smoke.txt"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 tools/prefill_bench.py 512 64 16 > "$OUT/prefill_prof.txt" 2>&1
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/prefill_kernel_stats.csv" \;
grep -E "B=" "$OUT/prefill_prof.txt"
