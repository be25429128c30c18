#!/bin/bash
# A/B measurement session into gpurun_out/$1: the GPU tests selected by $2 (-k expression, "" = all), then scripts/ubench32
# in mode $3 (skipped when empty), then one short bench line (no beside runs, no CPU baseline) per remaining argument
# "name:VAR=val ..." (empty var list = defaults).  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
rm -rf "$OUT" && mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > "$OUT/gputest.log" 2>&1 || exit 1
fi
if [ -n "$3" ]; then
  timeout -k 10 300 ./scripts/ubench32 $3 > "$OUT/ubench_$3.txt" 2>&1 || exit 1
fi
shift 3
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 300 python -u bench.py --beside-steps 0 --nomemo-steps 0 --cpu-sample 0 ${AB_ARGS:-} \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['ms_per_step'])" >> "$OUT/ab.txt"
done
exit 0
