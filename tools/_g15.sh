#!/bin/bash
# ORD (CPU-order GEMV) parity + A/B timing
set -o pipefail
O=gpurun_out/q3; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_ops_gpu.py -k "bit_exact or reference_outputs or baseline_configs or get_rows" > $O/pytest_mm.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpt2.py -k "quantized or logits_match" > $O/pytest_gpt2.log 2>&1 || exit 1
for ord in 1 0; do
  GGML_MI355X_MMV_ORDER=$ord timeout -k 10 300 python -u bench.py --no-cpu --no-gpt2 > $O/bench_ord$ord.json 2> $O/bench_ord$ord.err || exit 1
done
for t in q4_0 q8_0 q5_K; do for ord in 1 0; do
  GGML_MI355X_MMV_ORDER=$ord timeout -k 10 300 python -u bench.py --no-cpu --no-gpt2 --no-sweep --type $t > $O/bench_${t}_ord$ord.json 2>> $O/bench_ord.err || exit 1
done; done
