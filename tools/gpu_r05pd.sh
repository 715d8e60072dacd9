#!/bin/bash
# lone K >= 4096 decode GEMVs with every row of a wave in flight: parity + A/B against the old depth
set -eo pipefail
OUT=gpurun_out/${1:-r05pd}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_graphs_gpu.py > "$OUT/pytest.txt" 2>&1
tail -1 "$OUT/pytest.txt"
timeout -k 10 200 python3 -u tools/stamps.py lone q4_K:4096:4096:1 q4_K:4096:11008:1 q5_K:4096:4096:1 > "$OUT/lone_stamps.txt" 2>&1
for i in 1 2; do
  for v in 0 31; do
    GGML_MI355X_MMV_VARIANT=$v timeout -k 10 300 python3 -u bench.py --no-cpu --steps 20 > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); s=d['sweep']; print('variant $v', s['q4_K_4096x4096_single_graph']['us_per_mul_mat'], d['value'], s['q4_K_4096x11008']['GB/s'])"
  done
done
