#!/bin/bash
# The fp32 GPU tests against a build variant abvar/$1/libqlx.so, then the A/B bench of the main build against it
# (development tool).  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
QLX_LIB_PATH=abvar/$1/libqlx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_qnet32.py tests/test_gpu_qnet32_paths.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/$1.test.log 2>&1 || exit 1
export AB_ARGS="--steps 10 --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 --dp1-steps 0 --sparsity-steps 0"
bash scripts/ab_bench.sh "main:" "$1:QLX_LIB_PATH=abvar/$1/libqlx.so" "main_2:" "${1}_2:QLX_LIB_PATH=abvar/$1/libqlx.so"
