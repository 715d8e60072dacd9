#!/bin/bash
# bench.py without CPU legs or sweep (headline, prefill, GPT-2 decode / batched); prints the batched line
set -eo pipefail
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --no-cpu --no-sweep > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d.get('gpt2_batched'))"
