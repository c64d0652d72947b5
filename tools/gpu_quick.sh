# Usage: bash tools/gpu_quick.sh <tag>  -- GPU tests + GEMM shape bench + step bench (no profiler)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_$TAG.txt 2>&1; rc=$?
cat gpurun_out/gemm_$TAG.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json
exit $rc
