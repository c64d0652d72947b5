# Usage: bash tools/gpu_t.sh <tag> <pytest node ids...> -- selected GPU tests, then the GEMM shape bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-t}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread "$@" > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -25 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_$TAG.txt 2>&1; rc=$?
cat gpurun_out/gemm_$TAG.txt
exit $rc
