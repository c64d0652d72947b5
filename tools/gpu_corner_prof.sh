# Usage: bash tools/gpu_corner_prof.sh <tag> -- cornerNetCPool (BASELINE configs[3]) bench line + rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model cornerNetCPool --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cbench_$TAG.json 2> gpurun_out/cbench_$TAG.err || exit 1
cut -c1-300 gpurun_out/cbench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof_$TAG -o run -- python3 bench.py --model cornerNetCPool --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cprofbench_$TAG.json 2> gpurun_out/cprof_$TAG.err || exit 1
echo ok
# stall breakdown of the 64-channel layer1 GEMMs (register-staged conv_gemm_kernel<bf16,256,64>) and the layer2 ones
timeout -k 10 120 python tools/gemm_bench.py --only "layer1,layer2 3x3" > gpurun_out/gemm_l1_$TAG.txt 2>&1 || exit 1
cat gpurun_out/gemm_l1_$TAG.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/l1pmc_$TAG -o run -- python3 tools/gemm_bench.py --only "layer1" --reps 2 > /dev/null 2>&1 || exit 1
echo pmc ok
