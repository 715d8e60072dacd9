set -eo pipefail
for v in 4 12 20; do echo "mmq_variant $v"; GGML_MI355X_MMQ_VARIANT=$v PF_TYPES=q4_K,f16 timeout -k 10 120 python tools/prefill_bench.py 512 2>&1 | grep -v "^[EW]2026\|amdgpu.ids"; done
