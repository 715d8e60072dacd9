#!/bin/bash
# decode timelines: GPT-2 f16 / q4_k token stamps, batched step kernel trace
set -eo pipefail
OUT=gpurun_out/${1:-r05o}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/stamps.py gpt2 f16 8 > "$OUT/stamps_gpt2_f16.txt" 2>&1
timeout -k 10 120 python3 tools/stamps.py gpt2 q4_k 8 > "$OUT/stamps_gpt2_q4k.txt" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 tools/batched_prof.py > $OUT/prof_log.txt 2>&1
python3 tools/trace_summary.py $OUT/prof 62 8 > $OUT/batched_trace_summary.txt
cat $OUT/batched_trace_summary.txt | head -30
