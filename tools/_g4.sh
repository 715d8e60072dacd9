set -eo pipefail
mkdir -p gpurun_out/g4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 100 rocprofv3 --kernel-trace -d gpurun_out/g4/prof -o run --output-format csv -- python3 tools/micro_f16.py > gpurun_out/g4/order.json 2> gpurun_out/g4/err.txt
python3 tools/micro_f16.py --parse gpurun_out/g4/prof/run_kernel_trace.csv gpurun_out/g4/order.json
timeout -k 10 120 python tools/gpt2_prof.py 128 2>&1 | grep -v "^[EW]2026"
