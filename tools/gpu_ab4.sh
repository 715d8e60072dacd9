#!/bin/bash
# Round 4: headline kernel trace (no sweep), GEMV default candidates, k_mmqt split tiles
set -eo pipefail
OUT=gpurun_out/${1:-r04r}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu --no-gpt2 --no-sweep > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/headline_kernel_stats.csv" \;
head -3 "$OUT/headline_kernel_stats.csv" | cut -c1-200
for spec in "q4_K 4096 4096 32 21:0,31:0,21:2048,31:2048" "q4_K 4096 11008 14 21:0,31:0,21:2048,31:2048" "q5_K 4096 11008 12 11:0,21:0,21:2048,31:2048" "q4_0 4096 4096 36 22:0,32:0,22:768,32:768" "q8_0 4096 11008 8 21:0,11:0,11:2048"; do
  set -- $spec
  echo "== $1 ${2}x${3} R=$4" | tee -a $OUT/sweep.txt
  timeout -k 10 150 python3 -u tools/mmv_tune.py --variants $5 --rounds 9 --type $1 --K $2 --N $3 --rotate $4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/sweep.txt
done
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K PF_LONG=0,6,7,0,6,7 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf.txt
timeout -k 10 300 python -u -m pytest tests/test_prefill_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "split_k or bit_equal" > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
