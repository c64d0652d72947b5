# Usage: bash tools/gpu_gemmq.sh <tag> [only]  -- conv kernel tests with the ring kernel forced on, then
# gemm_bench on selected shapes with the ring kernel off (A) and on (B)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-gq}; ONLY=${2:-heads,deconv3,deconv2,layer3}
mkdir -p gpurun_out
SCD_GEMM_RING=1 SCD_WGRAD_RING=1 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv or deconv" > gpurun_out/gqk_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gqk_$TAG.log
[ $rc -eq 0 ] || exit $rc
SCD_GEMM_RING=0 timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/gqA_$TAG.txt 2>&1 || exit 1
SCD_GEMM_RING=1 timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/gqB_$TAG.txt 2>&1 || exit 1
paste gpurun_out/gqA_$TAG.txt gpurun_out/gqB_$TAG.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-60s | %s\n", $1, $2}'
