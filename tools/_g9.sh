set -eo pipefail
mkdir -p gpurun_out/g9
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0; do
echo "== mmq_variant $v"
GGML_MI355X_MMQ_VARIANT=$v PF_TYPES=q4_K python3 tools/pmc_kernel.py gpurun_out/g9/v$v k_mmq 'TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum' -- python3 tools/prefill_bench.py 512
done
