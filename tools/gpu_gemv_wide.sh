#!/bin/bash
# Round 4: Q4_0 / Q8_0 GEMV with 16-byte dword-aligned weight loads: mul_mat tests, the config-2/3
# sweep lines, and the Q4_0 counters again
set -eo pipefail
OUT=gpurun_out/${1:-r04wide}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mul_mat_gpu.py tests/test_00_reference_harness.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
for spec in "q4_0 4096 4096 36 12:0,22:0,32:0" "q8_0 4096 11008 8 11:0,21:0,31:0" "q4_K 4096 4096 32 31:0"; do
  set -- $spec
  echo "== $1 ${2}x${3} R=$4" | tee -a $OUT/sweep.txt
  timeout -k 10 150 python3 -u tools/mmv_tune.py --variants $5 --rounds 7 --type $1 --K $2 --N $3 --rotate $4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/sweep.txt
done
G="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE;TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
for spec in "q4_0 4096 4096 36 32:0" "q8_0 4096 11008 8 11:0"; do
  set -- $spec
  echo "== $1 ${2}x${3} variant $5" | tee -a $OUT/gemv_pmc.txt
  timeout -k 10 300 python3 -u tools/pmc_kernel.py $OUT/p_$1 k_mmv_stream "$G" -- python3 tools/mmv_tune.py --variants $5 --rounds 2 --type $1 --K $2 --N $3 --rotate $4 2>&1 | tee -a $OUT/gemv_pmc.txt
done
