set -o pipefail
mkdir -p gpurun_out/q4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/q4/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/q4/counters.txt | sort -u > gpurun_out/q4/sq.txt || true
export PF_TYPES=q4_K
timeout -k 10 300 python tools/pmc_kernel.py gpurun_out/q4/pmc k_mmqx "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE;SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" -- python3 tools/prefill_bench.py 512 > gpurun_out/q4/pmc.txt 2>&1
cat gpurun_out/q4/pmc.txt
