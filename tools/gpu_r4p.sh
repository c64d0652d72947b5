# Usage: bash tools/gpu_r4p.sh -- side stream CU budget (bench lines only: rocprofv3 kernel tracing crashed on the
# CU-masked queue), SQ counters of the stem kernels, and the Res50 narrow-ring re-test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_benchrr.sh sidecu "SCD_SIDE_CUS=0" "SCD_SIDE_CUS=128" "SCD_SIDE_CUS=96" "SCD_SIDE_CUS=64" || exit 1
bash tools/gpu_pmc_sq.sh stem "stem_" || exit 1
bash tools/gpu_r4o.sh || exit 1
echo r4p done
