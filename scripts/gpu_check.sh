set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/t_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --cpu-sample 0 > gpurun_out/bench_b1024.json 2> gpurun_out/bench_b1024.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --batch 256 --cpu-sample 0 > gpurun_out/bench_b256.json 2> gpurun_out/bench_b256.err || exit 1
