#!/bin/bash
# Quick GPU check into gpurun_out/$1 (default q): the GPU tests (optionally a -k filter in $2), smoke, then the default
# bench.  Every GPU step has its own time limit; the first failure ends the script (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-q}
rm -rf "$OUT" && mkdir -p "$OUT"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/gputest.log" 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
exit 0
