#!/bin/bash
# A/B: activation loads pinned ahead of the weight prefetch (default) vs compiler order (lib/ab)
set -eo pipefail
OUT=gpurun_out/${1:-r05ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for v in default ab; do
    if [ $v = ab ]; then export GGML_MI355X_BACKEND_LIB=$GRAFT_REPO_ROOT/ggml-imax_amd/lib/ab/libggml_mi355x.so; else unset GGML_MI355X_BACKEND_LIB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu --steps 20 > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.err"
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); s=d['sweep']; print('$v', d['value'], d['roofline']['frac'], s['q4_K_4096x4096_single_graph']['us_per_mul_mat'], s['q4_K_4096x11008']['GB/s'], s['q4_0_4096x4096']['GB/s'], s['q4_K_4096x4096_b64_prefill']['us_per_mul_mat_one_per_graph'], d['gpt2']['ms_per_decode_token'], d['gpt2_q4_k']['ms_per_decode_token'], d['gpt2_batched']['ms_per_step'])"
  done
done
