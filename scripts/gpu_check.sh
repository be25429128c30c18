#!/bin/bash
# One GPU session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.  Every GPU step has its own
# time limit and the script stops at the first failure of a GPU step (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/t_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
if [ "${QLX_PROFILE:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
    python3 bench.py --steps 10 --cpu-sample 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || exit 1
fi
exit 0
