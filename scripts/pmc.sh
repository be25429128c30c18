#!/bin/bash
# Hardware-counter passes (one counter group per rocprofv3 run; no trace domains with --pmc) over a short
# bench run, restricted to the update-path kernels.  Output: gpurun_out/pmc/<pass>/*_counter_collection.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
RE="${QLX_PMC_REGEX:-k_trunk|k_conv|k_gemm|k_bgemm|k_fc1|k_fc2|k_adam|k_update|k_slab|k_replay|k_env|k_sample|k_head|k_wreduce|k_slot}"
ARGS="--steps 2 --warmup 1 --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 --dp1-steps 0 --sparsity-steps 0 --cpu-sample 0 --profile-steps 1 ${QLX_PMC_ARGS:-}"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex "$RE" --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o c -- \
    python3 bench.py $ARGS > gpurun_out/pmc/$name.json 2> gpurun_out/pmc/$name.err
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run mix SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc > gpurun_out/pmc/traffic.log 2>&1
exit 0
