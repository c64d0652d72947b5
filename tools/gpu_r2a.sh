# Usage: bash tools/gpu_r2a.sh <tag> -- targeted GPU tests, 1-GPU bench, 2-rank self-launched bench rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-a}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ddp_gpu.py -x -v -k "bn_backward or world2" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
SCD_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err; rc=$?
cat gpurun_out/bench2_$TAG.json; tail -3 gpurun_out/bench2_$TAG.err
exit $rc
