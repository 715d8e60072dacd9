#!/bin/bash
# round 6 (session 2): repacked Q4_0 / short-prompt k_mmqt tests, then the k_mmqt threshold sweep
set -eo pipefail
OUT=gpurun_out/${1:-s2b}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_q40_repack_gpu.py tests/test_prefill_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for R in 2 4 8 16; do
  PF_TYPES=q4_K PF_R=$R PF_SINGLE=0 MMQ_VARIANTS=0 timeout -k 10 200 python -u tools/prefill_bench.py 48 64 96 128 > $OUT/pf_R$R.txt 2>&1
  GGML_MI355X_MMQT_SHORT=0 PF_TYPES=q4_K PF_R=$R PF_SINGLE=0 MMQ_VARIANTS=0 timeout -k 10 200 python -u tools/prefill_bench.py 48 64 96 128 > $OUT/pf_R${R}_off.txt 2>&1
  grep q4_K $OUT/pf_R$R.txt $OUT/pf_R${R}_off.txt
done
