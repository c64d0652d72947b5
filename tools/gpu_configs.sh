# Usage: bash tools/gpu_configs.sh <tag> -- the other BASELINE configs' bench lines (Res50 1024^2 B=16 fp16, cornerNetCPool
# B=32 bf16) and a rocprofv3 kernel trace of the cornerNetCPool step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cfg}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_${TAG}_res50.json 2> gpurun_out/bench_${TAG}_res50.err || exit 1
cut -c1-200 gpurun_out/bench_${TAG}_res50.json
timeout -k 10 300 python bench.py --model cornerNetCPool --no-cpu-baseline > gpurun_out/bench_${TAG}_corner.json 2> gpurun_out/bench_${TAG}_corner.err || exit 1
cut -c1-200 gpurun_out/bench_${TAG}_corner.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof_$TAG -o run -- python3 bench.py --model cornerNetCPool --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cprofbench_$TAG.json 2> gpurun_out/cprof_$TAG.err || exit 1
echo ok
