#!/bin/bash
# PMC passes over the bf16 GEMM core micro-benchmark (scripts/ubench_bgemm.hip, "pmc" mode: the fc1 forward at B = 1024 and
# at 8,192); one counter group per rocprofv3 run (MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC, <= 2 TA / TD / GRBM per pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcb}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-include-regex k_bgemm --pmc "$@" --output-format csv -d "$OUT/$name" -o c -- \
    ./scripts/ubench_bgemm 1024 pmc > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run mix SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run ta TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum || exit 1
exit 0
