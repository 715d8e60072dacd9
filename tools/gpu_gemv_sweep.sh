#!/bin/bash
# Round 4: the config-2/3 GEMVs (Q4_0 4096^2, Q4_K / Q5_K / Q8_0 4096 x 11008) over prefetch depth
# (mmv_variant tens digit) and grid size (mmv_blocks; 0 = resident count), interleaved in one process
set -eo pipefail
OUT=gpurun_out/${1:-r04o}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "q4_0 4096 4096 36 12:0,22:0,32:0,22:768,22:1536,22:2048" "q4_K 4096 11008 14 11:0,21:0,31:0,21:768,21:1536,21:2048" "q5_K 4096 11008 12 11:0,21:0,31:0,11:768,11:1536,11:2048" "q8_0 4096 11008 8 11:0,21:0,31:0,21:1536"; do
  set -- $spec
  echo "== $1 ${2}x${3} R=$4" | tee -a $OUT/sweep.txt
  timeout -k 10 150 python3 -u tools/mmv_tune.py --variants $5 --rounds 7 --type $1 --K $2 --N $3 --rotate $4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/sweep.txt
done
