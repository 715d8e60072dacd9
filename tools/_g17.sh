#!/bin/bash
set -o pipefail
O=gpurun_out/q5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gguf.py > $O/pytest_gguf.log 2>&1 || exit 1
for t in q4_K q4_0; do for ord in 0 1 2; do
  GGML_MI355X_MMV_ORDER=$ord timeout -k 10 300 python -u bench.py --no-cpu --no-gpt2 --no-sweep --type $t > $O/bench_${t}_ord$ord.json 2>> $O/bench.err || exit 1
done; done
