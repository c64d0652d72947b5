# Usage: bash tools/gpu_envab.sh <tag> <VAR> [only]  -- conv/heads kernel tests with VAR=1, then gemm_bench with
# VAR=0 (A) and VAR=1 (B), twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; ONLY=${3:-heads,deconv3,deconv2,layer3,layer4}
mkdir -p gpurun_out
env $VAR=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv or deconv or heads" --timeout 120 --timeout-method thread > gpurun_out/eab_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/eab_$TAG.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  env $VAR=0 timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/eabA_$TAG.txt 2>&1 || exit 1
  env $VAR=1 timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 > gpurun_out/eabB_$TAG.txt 2>&1 || exit 1
  paste gpurun_out/eabA_$TAG.txt gpurun_out/eabB_$TAG.txt | grep -v amdgpu.ids | grep -v wgrad
done
