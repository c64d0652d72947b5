# Usage: bash tools/gpu_heads.sh <tag> -- heads GEMM parity tests, standalone GEMM timing, 1-GPU bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-h}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bf16_parity_gpu.py -x -q -k "heads or groups" --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gemm_bench.py --only heads > gpurun_out/gemm_$TAG.log 2>&1; rc=$?
cat gpurun_out/gemm_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json
exit $rc
