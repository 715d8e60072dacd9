#!/bin/bash
# Scratch A/B (round 4): nontemporal weight loads in the streaming GEMV (mmv_variant + 100) on the
# headline and the sweep shapes; per-node timer test; LLaMA block test
set -eo pipefail
OUT=gpurun_out/${1:-r04g}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "q4_K 4096 4096 32" "q4_0 4096 4096 36" "q4_K 4096 11008 14" "q5_K 4096 11008 12" "q8_0 4096 11008 8"; do
  set -- $spec
  echo "== $1 ${2}x${3} R=$4" | tee -a $OUT/nt.txt
  timeout -k 10 120 python3 -u tools/mmv_tune.py --variants 0:0,100:0 --rounds 9 --type $1 --K $2 --N $3 --rotate $4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/nt.txt
done
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_llama_block_gpu.py tests/test_prefill_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "per_node or llama or bit_equal" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
grep -E "PASS|FAIL|T=|launches" $OUT/pytest.log | tail -12
