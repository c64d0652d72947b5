# Usage: bash tools/gpu_ablate.sh <only> [variants]  -- gemm_bench over the compile-time ablation builds
# (make -C scd-resnet_amd/csrc ablate ABLATE=N beforehand; 0 = the product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=${1:-heads}; VARS=${2:-0 1 2 3 4 5 0}
for V in $VARS; do
  if [ "$V" = 0 ]; then L=scd-resnet_amd/scdhip/libscdhip.so; else L=scd-resnet_amd/scdhip/libscdhip_ablate$V.so; fi
  echo "== ablate $V"
  SCDHIP_LIB=$PWD/$L timeout -k 10 120 python tools/gemm_bench.py --only $ONLY --reps 20 2>&1 | grep -E "fwd|dgrad|wgrad" || exit 1
done
