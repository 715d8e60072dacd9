set -eo pipefail
mkdir -p gpurun_out/g10
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g10/split.log 2>&1 || { tail -40 gpurun_out/g10/split.log; exit 1; }
tail -3 gpurun_out/g10/split.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g10/all.log 2>&1 || { tail -40 gpurun_out/g10/all.log; exit 1; }
tail -3 gpurun_out/g10/all.log
