set -eo pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K,q5_K PF_LONG=1,2 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf_long.txt
