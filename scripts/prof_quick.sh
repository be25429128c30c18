#!/bin/bash
# Quick per-kernel timing + HBM fetch of a short bench run: one --kernel-trace --stats pass and one FETCH_SIZE
# pass (separate runs, no trace domains with --pmc).  Output: gpurun_out/pq/{stats,fetch}/..., summary.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/pq && mkdir -p gpurun_out/pq
ARGS="--steps ${QLX_PQ_STEPS:-3} --warmup 1 --beside-steps 0 --cpu-sample 0 --profile-steps 1 ${QLX_PQ_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq/stats -o s -- \
  python3 bench.py $ARGS > gpurun_out/pq/stats.json 2> gpurun_out/pq/stats.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-include-regex "${QLX_PMC_REGEX:-k_}" --pmc FETCH_SIZE --output-format csv \
  -d gpurun_out/pq/fetch -o f -- python3 bench.py $ARGS > gpurun_out/pq/fetch.json 2> gpurun_out/pq/fetch.err || exit 1
python3 scripts/prof_summary.py gpurun_out/pq > gpurun_out/pq/summary.txt 2>&1
exit 0
