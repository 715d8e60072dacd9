#!/bin/bash
# Round 4 quick check: graph-capture and GPT-2 GPU tests, then the bench without CPU legs or sweep
set -eo pipefail
OUT=gpurun_out/${1:-r04y}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_gpt2.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu --no-sweep > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic_source']['file'], d.get('gpt2_batched'))"
