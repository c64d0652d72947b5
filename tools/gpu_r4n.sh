# Usage: bash tools/gpu_r4n.sh -- the weight-gradient side stream confined to part of the chip (SCD_SIDE_CUS = 0 /
# 192 / 128 CUs) A/B, then SQ counters of the stem kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_abn.sh sidecu "SCD_SIDE_CUS=0" "SCD_SIDE_CUS=192" "SCD_SIDE_CUS=128" || exit 1
bash tools/gpu_pmc_sq.sh stem "stem_" || exit 1
echo r4n done
