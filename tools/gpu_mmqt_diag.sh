#!/bin/bash
# Round 4: k_mmqt phase stamps and timing ablations (diagnostic build lib/diag; results invalid)
set -eo pipefail
OUT=gpurun_out/${1:-r04l}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GGML_MI355X_BACKEND_LIB=$GRAFT_REPO_ROOT/ggml-imax_amd/lib/diag/libggml_mi355x.so
for A in 0 1 2 4 6; do
  echo "== ablation $A" | tee -a $OUT/stamps.txt
  timeout -k 10 120 python3 -u tools/mmqt_stamps.py 512 $A 2>&1 | grep --line-buffered -v amdgpu.ids | tee -a $OUT/stamps.txt
done
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K PF_LONG=0,16,17,18,20,22 MMQ_VARIANTS=0 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/abl_timing.txt
