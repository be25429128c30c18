#!/bin/bash
# Copy one scripts/profile_round.sh output (gpurun_out/<name>) into profiles/<name>: the bench line, logs, the rocprofv3
# kernel statistics with a per-kernel summary (+ FETCH_SIZE per dispatch), the PMC summary and the per-scope HBM traffic.
set -e
cd "$(dirname "$0")/.."
name=$1
src=gpurun_out/$name
dst=profiles/$name
mkdir -p "$dst"
cp "$src/bench.json" "$src/bench.err" "$src/gputest.log" "$dst/"
cp "$(ls $src/stats/*kernel_stats.csv | head -1)" "$dst/kernel_stats.csv"
mkdir -p /tmp/collect_$name && rm -rf /tmp/collect_$name/* && cp -r "$src/stats" /tmp/collect_$name/stats && cp -r "$src/pmc/fetch" /tmp/collect_$name/fetch
python3 scripts/prof_summary.py /tmp/collect_$name > "$dst/rocprof_summary.txt"
python3 scripts/pmc_summary.py "$src/pmc" > "$dst/pmc_summary.txt"
cp "$src/pmc/pmc_traffic_fp32.json" "$dst/pmc_traffic_fp32.json" 2>/dev/null || python3 scripts/pmc_traffic.py "$src/pmc" fp32 > /dev/null
[ -f "$dst/pmc_traffic_fp32.json" ] || cp "$src/pmc/pmc_traffic_fp32.json" "$dst/"
ls "$dst"
