set -o pipefail
mkdir -p gpurun_out/q2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K,q5_K
timeout -k 10 120 python -u tools/prefill_bench.py 512 64 16 > gpurun_out/q2/new.txt 2>&1
GGML_MI355X_MMQ_VARIANT=64 timeout -k 10 120 python -u tools/prefill_bench.py 512 64 > gpurun_out/q2/xcd.txt 2>&1
GGML_MI355X_MMQ_VARIANT=32 timeout -k 10 120 python -u tools/prefill_bench.py 512 64 > gpurun_out/q2/old.txt 2>&1
PF_TYPES=q4_K timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/q2/prof -o run --output-format csv -- python3 tools/prefill_bench.py 512 64 > gpurun_out/q2/prof.txt 2>&1
find gpurun_out/q2/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/q2/kernel_stats.csv \;
cat gpurun_out/q2/new.txt gpurun_out/q2/xcd.txt gpurun_out/q2/old.txt
python tools/kstats.py gpurun_out/q2/kernel_stats.csv 8
