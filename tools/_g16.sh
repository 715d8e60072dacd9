#!/bin/bash
set -o pipefail
O=gpurun_out/q4; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mul_mat_gpu.py tests/test_ops_gpu.py > $O/pytest_mm.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpt2.py -k "quantized or logits_match" > $O/pytest_gpt2.log 2>&1 || exit 1
