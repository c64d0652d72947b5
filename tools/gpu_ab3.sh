# Usage: bash tools/gpu_ab3.sh <tag> [only]  -- conv/heads kernel tests, then gemm_bench with the baseline library
# (scdhip/libscdhip_base.so, A) and the current one (B)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ab}; ONLY=${2:-heads,deconv3,deconv2,layer3,layer4,layer2}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abk_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/abk_$TAG.log
[ $rc -eq 0 ] || exit $rc
SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_base.so timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/abA_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/abB_$TAG.txt 2>&1 || exit 1
paste gpurun_out/abA_$TAG.txt gpurun_out/abB_$TAG.txt | grep -v amdgpu.ids
