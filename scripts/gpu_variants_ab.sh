#!/bin/bash
# Parity of the main build's fp32 paths, then bench.py A/B of the main build against build variants abvar/<v>/libqlx.so
# (development tool; one JSON line each in gpurun_out/ab/).  Usage: gpu_variants_ab.sh v1 v2 ...  Every GPU step has its
# own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_qnet32.py tests/test_gpu_qnet32_paths.py ${AB_TESTS:-} -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/ab/main.test.log 2>&1 || exit 1
export AB_ARGS="--steps 10 --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 --dp1-steps 0 --sparsity-steps 0"
specs=("main:")
for v in "$@"; do specs+=("$v:QLX_LIB_PATH=abvar/$v/libqlx.so"); done
specs+=("main_2:")
for v in "$@"; do specs+=("${v}_2:QLX_LIB_PATH=abvar/$v/libqlx.so"); done
bash scripts/ab_bench.sh "${specs[@]}"
