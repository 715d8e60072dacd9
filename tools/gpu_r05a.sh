#!/bin/bash
# Round-5 baseline: dependent-kernel floors, lone GEMV per graph (host + device), Q4_K GPT-2 decode trace
set -eo pipefail
OUT=gpurun_out/${1:-r05a}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 tools/kfloor > "$OUT/kfloor.txt" 2>&1
cat "$OUT/kfloor.txt"
CASES="q4_K:4096:4096:1 q4_K:4096:11008:1 q4_K:768:2304:1 q4_K:3072:768:1 q4_0:4096:4096:1 f16:768:2304:1 q4_K:4096:4096:8 q4_K:4096:4096:64"
timeout -k 10 200 python3 -u tools/lone_gemv.py $CASES > "$OUT/lone.txt" 2>&1
cat "$OUT/lone.txt"
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/prof_lone" -o run --output-format csv -- python3 tools/lone_gemv.py $CASES > "$OUT/lone_prof.txt" 2>&1
python3 tools/ktrace.py "$(find $OUT/prof_lone -name '*kernel_trace.csv' | head -1)" > "$OUT/lone_ktrace.txt"
cat "$OUT/lone_ktrace.txt"
GPT2_QTYPE=q4_k bash tools/gpt2_trace.sh "${1:-r05a}/gpt2q4k_trace" 62 | tail -14
bash tools/gpt2_trace.sh "${1:-r05a}/gpt2f16_trace" 50 | tail -12
