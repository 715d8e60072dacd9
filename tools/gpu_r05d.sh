#!/bin/bash
# kernel-argument placement A/B (HIP_FORCE_DEV_KERNARG) on the dependent-kernel floor, lone GEMVs and GPT-2 decode
set -eo pipefail
OUT=gpurun_out/${1:-r05d}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for KA in 0 1; do
  echo "== HIP_FORCE_DEV_KERNARG=$KA"
  HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 100 tools/kfloor > "$OUT/kfloor_ka$KA.txt" 2>&1; head -4 "$OUT/kfloor_ka$KA.txt"
  HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 200 python3 -u tools/lone_gemv.py q4_K:4096:4096:1 q4_K:768:2304:1 f16:768:2304:1 > "$OUT/lone_ka$KA.txt" 2>&1; cat "$OUT/lone_ka$KA.txt"
  HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 200 python3 -u tools/gpt2_prof.py 64 > "$OUT/gpt2_ka$KA.txt" 2>&1; grep tok/s "$OUT/gpt2_ka$KA.txt"
  HIP_FORCE_DEV_KERNARG=$KA GPT2_QTYPE=q4_k timeout -k 10 200 python3 -u tools/gpt2_prof.py 64 > "$OUT/gpt2q_ka$KA.txt" 2>&1; grep tok/s "$OUT/gpt2q_ka$KA.txt"
  HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 200 python3 -u tools/stamps.py gpt2 f16 8 > "$OUT/stamps_f16_ka$KA.txt" 2>&1; tail -2 "$OUT/stamps_f16_ka$KA.txt"
done
