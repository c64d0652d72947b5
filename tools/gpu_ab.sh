# Usage: bash tools/gpu_ab.sh <tag> <ENVVAR>  -- kernel tests with ENVVAR=1, then gemm_bench and bench
# with ENVVAR=0 and with the default choice (A/B of a kernel variant in one call).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ab}; VAR=${2:-SCD_GEMM_RING}
mkdir -p gpurun_out
env $VAR=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abk_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/abk_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
env $VAR=0 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemmA_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemmB_$TAG.txt 2>&1 || exit 1
paste gpurun_out/gemmA_$TAG.txt gpurun_out/gemmB_$TAG.txt | awk -F'\t' '{printf "%-60s | %s\n", $1, $2}'
env $VAR=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/benchA_$TAG.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/benchB_$TAG.json 2>/dev/null || exit 1
cut -c1-200 gpurun_out/benchA_$TAG.json gpurun_out/benchB_$TAG.json
