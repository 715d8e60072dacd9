set -eo pipefail
timeout -k 10 300 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/g11.log 2>&1 || { tail -40 gpurun_out/g11.log; exit 1; }
tail -3 gpurun_out/g11.log
