#!/bin/bash
# One A/B session into gpurun_out/$1: the GPU tests selected by $2 (-k expression; "" = skip), then one short bench line
# per remaining argument "name:VAR=val ..." (A/B of environment switches or QLX_LIB_PATH variant builds), each repeated
# twice in alternating order.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
rm -rf "$OUT" && mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > "$OUT/gputest.log" 2>&1 || exit 1
fi
shift 2
for rep in a b; do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 300 python -u bench.py --beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 \
      --dp1-steps 0 --c5-steps 0 --cpu-sample 0 ${AB_ARGS:-} > "$OUT/$name$rep.json" 2> "$OUT/$name$rep.err" || exit 1
    python3 -c "import json;d=json.load(open('$OUT/$name$rep.json'));print('$name$rep', d['value'], d['ms_per_step'])" >> "$OUT/ab.txt"
  done
done
exit 0
