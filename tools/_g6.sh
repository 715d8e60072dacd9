set -eo pipefail
mkdir -p gpurun_out/g6
timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g6/pytest.log 2>&1 || { tail -30 gpurun_out/g6/pytest.log; exit 1; }
tail -2 gpurun_out/g6/pytest.log
for v in 1 0; do echo "mmq_variant $v"; GGML_MI355X_MMQ_VARIANT=$v PF_TYPES=q4_K,q8_0,f16 timeout -k 10 120 python tools/prefill_bench.py 512 64 2>&1 | grep -v "^[EW]2026"; done
