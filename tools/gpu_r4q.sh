# Usage: bash tools/gpu_r4q.sh -- weight-gradient split counts re-tuned on the fixed GEMMs (bench lines only): the
# reduce's slab pricing (SCD_WGRAD_SLAB_TBPS, lower = fewer splits), the layer1 weight gradient's split cap, and the
# narrow 1x1 ring routing on the Res10 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_benchrr.sh slab "SCD_WGRAD_SLAB_TBPS=0.8" "SCD_WGRAD_SLAB_TBPS=0.4" "SCD_WGRAD_SLAB_TBPS=1.6" "SCD_WGRAD_L1_NSPLIT=64" "SCD_GEMM_NARROW_RING=1" || exit 1
echo r4q done
