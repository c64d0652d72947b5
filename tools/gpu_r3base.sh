# Usage: bash tools/gpu_r3base.sh <tag> -- round-3 baseline: bench eager + graph, host overhead, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-b}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-300 gpurun_out/bench_$TAG.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/benchg_$TAG.json 2> gpurun_out/benchg_$TAG.err || exit 1
cut -c1-300 gpurun_out/benchg_$TAG.json
timeout -k 10 300 python tools/host_overhead.py > gpurun_out/host_$TAG.txt 2>&1 || exit 1
tail -5 gpurun_out/host_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
find gpurun_out/prof_$TAG -name "*.csv" | head
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_ddp_gpu.py "tests/test_corner_gpu.py::test_shared_feature_gradient_with_extra_consumer" > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/tests_$TAG.log
exit $rc
