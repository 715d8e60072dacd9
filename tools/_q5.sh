set -o pipefail
mkdir -p gpurun_out/q5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PF_TYPES=q4_K
for v in 0 256 512 768 1024 1792; do
  echo "variant $v" >> gpurun_out/q5/abl.txt
  GGML_MI355X_MMQ_VARIANT=$v timeout -k 10 120 python -u tools/prefill_bench.py 512 16 2>&1 | grep -v amdgpu.ids >> gpurun_out/q5/abl.txt
done
cat gpurun_out/q5/abl.txt
