#!/bin/bash
# A/B bench of environment-variable variants (development tool): one bench.py run per variant, one JSON line
# each in gpurun_out/ab/<name>.json.  Usage: ab_bench.sh "name:VAR=val VAR2=val" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python bench.py --cpu-sample 0 ${AB_ARGS:-} > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));print('$name', d['value'], d['ms_per_step'])"
done
exit 0
