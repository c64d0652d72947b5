# Usage: bash tools/gpu_h384.sh <tag> <variant libs...> -- heads GEMM tests, heads rows of gemm_bench per variant, step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "heads or F1 or f1" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh heads 20 "$@" > gpurun_out/var_$TAG.txt 2>&1 || { tail gpurun_out/var_$TAG.txt; exit 1; }
cat gpurun_out/var_$TAG.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cut -c1-150 gpurun_out/bench_$TAG.json; python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['roofline'])"
exit $rc
