# Usage: bash tools/gpu_ablate.sh <tag> <only> -- gemm_bench with the ring GEMM ablations (SCD_GEMM_DEBUG 0/1/2)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-abl}; ONLY=${2:-heads}
mkdir -p gpurun_out
for D in 0 1 2; do
  echo "== SCD_GEMM_DEBUG=$D"
  SCD_GEMM_RING=1 SCD_GEMM_DEBUG=$D timeout -k 10 300 python tools/gemm_bench.py --only $ONLY --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
done
