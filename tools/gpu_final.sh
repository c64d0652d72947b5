# Usage: bash tools/gpu_final.sh <tag> -- round measurements without the test suite: bench (with CPU baseline),
# rocprofv3 kernel stats of the same bench command, the two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic,
# and the other BASELINE configs' bench lines (Res50 1024^2 B=16 fp16, cornerNetCPool B=32 bf16)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-220 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$TAG.json 2> gpurun_out/pmcf_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw_$TAG.json 2> gpurun_out/pmcw_$TAG.err || exit 1
timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --no-cpu-baseline > gpurun_out/bench_${TAG}_res50.json 2> gpurun_out/bench_${TAG}_res50.err || exit 1
cut -c1-200 gpurun_out/bench_${TAG}_res50.json
timeout -k 10 300 python bench.py --model cornerNetCPool --no-cpu-baseline > gpurun_out/bench_${TAG}_corner.json 2> gpurun_out/bench_${TAG}_corner.err || exit 1
cut -c1-200 gpurun_out/bench_${TAG}_corner.json
find gpurun_out/prof_$TAG gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG -name "*.csv" | head -20
