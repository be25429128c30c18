#!/bin/bash
# One round's measurement set into gpurun_out/$1 (default r): the GPU test suite, smoke, the headline bench (fp32 C3 with
# the per-batch-target / dense-frame / reference-work / single-rank-DP figures, bf16 beside and the CPU baseline in the same
# line), rocprofv3 --kernel-trace --stats passes of the fp32 and the bf16 loop, the PMC traffic passes of scripts/pmc.sh for
# both precisions, the bf16 GEMM-core micro-benchmark and the full 10,000-step C1 CPU baseline.  Every GPU step has its own
# time limit; the first failure ends the script.  Part (second argument) a = tests, smoke, bench, rocprof stats;
# b = PMC passes, micro-benchmark, CPU baseline; default both (two gpurun calls keep each under the call limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r}
PART=${2:-ab}
mkdir -p "$OUT"
SHORT="--steps 3 --warmup 1 --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 --dp1-steps 0 --sparsity-steps 0 --cpu-sample 0 --profile-steps 1"
if [[ $PART == *a* ]]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o s -- \
  python3 bench.py $SHORT > "$OUT/stats.json" 2> "$OUT/stats.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_bf16" -o s -- \
  python3 bench.py --precision bf16 $SHORT > "$OUT/stats_bf16.json" 2> "$OUT/stats_bf16.err" || exit 1
fi
if [[ $PART == *b* ]]; then
bash scripts/pmc.sh || exit 1
rm -rf "$OUT/pmc" && mv gpurun_out/pmc "$OUT/pmc"
python3 scripts/pmc_traffic.py "$OUT/pmc" fp32 > "$OUT/pmc_traffic.log" 2>&1
QLX_PMC_ARGS="--precision bf16" bash scripts/pmc.sh || exit 1
rm -rf "$OUT/pmc_bf16" && mv gpurun_out/pmc "$OUT/pmc_bf16"
python3 scripts/pmc_traffic.py "$OUT/pmc_bf16" bf16 > "$OUT/pmc_traffic_bf16.log" 2>&1
timeout -k 10 200 ./scripts/ubench_bgemm > "$OUT/ubench_bgemm.txt" 2>&1 || exit 1
timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.cpu_baseline(10000)))" > "$OUT/cpu_full.json" 2>&1 || exit 1
# the per-dispatch counter tables exceed what gpurun copies back (64 MiB): compressed here, gunzip before collect_profile.sh
find "$OUT" -name '*.csv' -size +512k -exec gzip -f {} +
fi
exit 0
