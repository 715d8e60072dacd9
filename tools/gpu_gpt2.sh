#!/bin/bash
# GPT-2 checks: driver tests (parity, CLI, launch counts) + decode timing with/without host I/O
set -eo pipefail
OUT=gpurun_out/${1:-gpt2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpt2.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for h in 1 0 1; do
  GPT2_HOST_IO=$h timeout -k 10 120 python -u tools/gpt2_prof.py 128 > "$OUT/gpt2_prof_h$h.log" 2>&1
  echo "host_io=$h"; cat "$OUT/gpt2_prof_h$h.log"
done
