#!/bin/bash
# Copy one scripts/profile_round.sh output (gpurun_out/<name>) into profiles/<name>: the bench line, logs, the rocprofv3
# kernel statistics of the fp32 and the bf16 loop with per-kernel summaries (+ FETCH_SIZE per dispatch), the PMC summary,
# the per-scope HBM traffic of both precisions, the bf16 GEMM-core micro-benchmark and the full C1 CPU baseline.
set -e
cd "$(dirname "$0")/.."
name=$1
src=gpurun_out/$name
dst=profiles/$name
mkdir -p "$dst"
find "$src" -name '*.csv.gz' -exec gunzip -f {} +
cp "$src/bench.json" "$src/bench.err" "$src/gputest.log" "$src/smoke.log" "$dst/"
cp "$(ls $src/stats/*kernel_stats.csv | head -1)" "$dst/kernel_stats.csv"
cp "$(ls $src/stats_bf16/*kernel_stats.csv | head -1)" "$dst/kernel_stats_bf16.csv"
for p in "" _bf16; do
  t=/tmp/collect_$name$p
  mkdir -p $t && rm -rf $t/* && cp -r "$src/stats$p" $t/stats && cp -r "$src/pmc$p/fetch" $t/fetch
  python3 scripts/prof_summary.py $t > "$dst/rocprof_summary$p.txt"
done
python3 scripts/pmc_summary.py "$src/pmc" > "$dst/pmc_summary.txt"
cp "$src/pmc/pmc_traffic_fp32.json" "$dst/pmc_traffic_fp32.json"
cp "$src/pmc_bf16/pmc_traffic_bf16.json" "$dst/pmc_traffic_bf16.json"
cp "$src/ubench_bgemm.txt" "$src/cpu_full.json" "$dst/" 2>/dev/null || true
ls "$dst"
