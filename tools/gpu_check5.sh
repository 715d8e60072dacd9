#!/bin/bash
# Round 4 check: the fused canonical fold (every Q4_K / Q5_K prefill kernel) and the direct-launch
# rule for streaming topologies -- prefill / graphs / GPT-2 GPU tests, prefill timing, bench
set -eo pipefail
OUT=gpurun_out/${1:-r04v}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_prefill_gpu.py tests/test_graphs_gpu.py tests/test_gpt2.py tests/test_llama_block_gpu.py tests/test_mul_mat_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; tail -1 $OUT/pytest.log; exit 1; }
PF_SINGLE=0 PF_R=16 PF_TYPES=q4_K,q5_K MMQ_VARIANTS=0 PF_LONG=0,1 timeout -k 10 300 python3 -u tools/prefill_bench.py 512 256 64 2>&1 | grep --line-buffered -v amdgpu.ids | tee $OUT/pf.txt
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['sweep']['q4_K_4096x4096_b512_prefill']['us_per_mul_mat'], d.get('gpt2_batched'))"
