set -o pipefail
mkdir -p gpurun_out/q1
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py tests/test_mul_mat_gpu.py -x -v --timeout 120 --timeout-method thread -k "prefill or b_q4 or b_q5 or shapes" > gpurun_out/q1/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/q1/pytest.log
exit $rc
