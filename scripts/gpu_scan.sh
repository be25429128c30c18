#!/bin/bash
# GPU tests + bench + profile (gpu_check.sh), then a rocprofv3 kernel trace of the trunk batch scan.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scan -o scan -- \
  python3 scripts/trunk_scan.py > gpurun_out/scan.log 2>&1 || exit 1
exit 0
