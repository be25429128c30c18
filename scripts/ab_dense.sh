#!/bin/bash
# A/B of the dense-variable update on the aux stream (QLX_F32_DENSE_OVERLAP): the fp32 bit-exact tests with it on, then the
# fp32 C3 bench with it off / on / off / on (headline loop only), every GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}
mkdir -p "$OUT"
QLX_F32_DENSE_OVERLAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_qnet32.py tests/test_gpu_learner.py tests/test_gpu_per.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > "$OUT/gputest_overlap.log" 2>&1 || exit 1
ARGS="--beside-steps 0 --nomemo-steps 0 --dense-steps 0 --refwork-steps 0 --dp1-steps 0 --cpu-sample 0 --steps 20"
for i in 1 2; do
  QLX_F32_DENSE_OVERLAP=0 timeout -k 10 150 python -u bench.py $ARGS > "$OUT/off$i.json" 2> "$OUT/off$i.err" || exit 1
  QLX_F32_DENSE_OVERLAP=1 timeout -k 10 150 python -u bench.py $ARGS > "$OUT/on$i.json" 2> "$OUT/on$i.err" || exit 1
done
exit 0
