#!/bin/bash
# Round-5 phase stamps (diagnostic build): lone GEMVs and the GPT-2 decode token timeline
set -eo pipefail
OUT=gpurun_out/${1:-r05b}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u tools/stamps.py lone q4_K:4096:4096:1 q4_K:768:2304:1 q4_K:3072:768:1 q4_0:4096:4096:1 f16:768:2304:1 > "$OUT/lone.txt" 2>&1
cat "$OUT/lone.txt"
timeout -k 10 200 python3 -u tools/stamps.py gpt2 f16 8 > "$OUT/gpt2_f16.txt" 2>&1
cat "$OUT/gpt2_f16.txt"
timeout -k 10 200 python3 -u tools/stamps.py gpt2 q4_k 8 > "$OUT/gpt2_q4k.txt" 2>&1
cat "$OUT/gpt2_q4k.txt"
