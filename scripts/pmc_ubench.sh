#!/bin/bash
# PMC passes over the kernel micro-benchmark (GEMM section); one counter group per rocprofv3 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcu
RE="${QLX_PMC_REGEX:-k_gemm}"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RE" --pmc "$@" --output-format csv -d gpurun_out/pmcu/$name -o c -- \
    ./scripts/ubench ${QLX_UB_MODE:-gemm} > gpurun_out/pmcu/$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run mix SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmcu > gpurun_out/pmcu/summary.txt 2>&1
exit 0
