#!/bin/bash
# One round's measurement set into gpurun_out/$1 (default r): the GPU test suite, the headline bench (fp32 C3 with the
# per-batch-target figure, bf16 beside and the CPU baseline in the same line), a rocprofv3 --kernel-trace --stats pass
# and the PMC passes of scripts/pmc.sh.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r}
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o s -- \
  python3 bench.py --steps 3 --warmup 1 --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --sparsity-steps 0 --cpu-sample 0 --profile-steps 1 > "$OUT/stats.json" \
  2> "$OUT/stats.err" || exit 1
bash scripts/pmc.sh || exit 1
mv gpurun_out/pmc "$OUT/pmc"
python3 scripts/pmc_traffic.py "$OUT/pmc" fp32 > "$OUT/pmc_traffic.log" 2>&1
exit 0
