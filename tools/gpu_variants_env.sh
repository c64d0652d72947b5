# Usage: bash tools/gpu_variants_env.sh <only> <reps> <"ENV=V ..." settings...> -- gemm_bench rows per environment setting
set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=$1; shift; REPS=$1; shift
for round in 1 2; do
  for v in "$@"; do
    echo "== $v (round $round)"
    env $v timeout -k 10 120 python tools/gemm_bench.py --only "$ONLY" --reps $REPS 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
