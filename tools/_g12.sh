set -eo pipefail
mkdir -p gpurun_out/g12
timeout -k 10 400 python -u -m pytest tests/test_gpt2.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g12/pytest.log 2>&1 || { tail -30 gpurun_out/g12/pytest.log; exit 1; }
tail -2 gpurun_out/g12/pytest.log
for v in 1 0; do GGML_MI355X_ATTN_VARIANT=$v timeout -k 10 120 python tools/gpt2_prof.py 128 2>&1 | grep -v "^[EW]2026"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g12/prof -o run --output-format csv -- python3 tools/gpt2_prof.py 64 > /dev/null 2>&1
python3 tools/kstats.py gpurun_out/g12/prof/run_kernel_stats.csv 8
