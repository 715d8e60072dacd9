set -eo pipefail
mkdir -p gpurun_out/g14
timeout -k 10 400 python -u -m pytest tests/test_gpt2.py tests/test_ops_gpu.py tests/test_mul_mat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g14/pytest.log 2>&1 || { tail -30 gpurun_out/g14/pytest.log; exit 1; }
tail -2 gpurun_out/g14/pytest.log
timeout -k 10 120 python tools/gpt2_prof.py 128 2>&1 | grep -v "^[EW]2026"
