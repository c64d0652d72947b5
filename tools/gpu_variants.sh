# Usage: bash tools/gpu_variants.sh <only> <reps> <lib names...> -- gemm_bench rows for each variant library, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=$1; shift; REPS=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then LIBP=""; else LIBP=scd-resnet_amd/scdhip/libscdhip_$v.so; fi
    echo "== $v (round $round)"
    SCDHIP_LIB=${LIBP:-scd-resnet_amd/scdhip/libscdhip.so} timeout -k 10 120 python tools/gemm_bench.py --only "$ONLY" --reps $REPS 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
