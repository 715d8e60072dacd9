set -o pipefail
mkdir -p gpurun_out/q3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K,q5_K
timeout -k 10 200 python -u -m pytest tests/test_prefill_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q3/pytest.log 2>&1
tail -3 gpurun_out/q3/pytest.log
GGML_MI355X_MMQ_VARIANT=128 timeout -k 10 200 python -u -m pytest tests/test_prefill_gpu.py -x -q --timeout 120 --timeout-method thread -k "shapes or edge or sharded" > gpurun_out/q3/pytest_sk2.log 2>&1
tail -3 gpurun_out/q3/pytest_sk2.log
timeout -k 10 120 python -u tools/prefill_bench.py 512 64 16 > gpurun_out/q3/sk1.txt 2>&1
GGML_MI355X_MMQ_VARIANT=64 timeout -k 10 120 python -u tools/prefill_bench.py 512 64 > gpurun_out/q3/sk1xcd.txt 2>&1
GGML_MI355X_MMQ_VARIANT=128 timeout -k 10 120 python -u tools/prefill_bench.py 512 64 > gpurun_out/q3/sk2.txt 2>&1
cat gpurun_out/q3/sk1.txt gpurun_out/q3/sk1xcd.txt gpurun_out/q3/sk2.txt | grep -v amdgpu.ids
