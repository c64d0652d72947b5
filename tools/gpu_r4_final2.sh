# Usage: bash tools/gpu_r4_final2.sh [tag] -- the round's PMC HBM-traffic passes and configs[3]/[4] bench lines +
# kernel traces (tools/gpu_r3_profiles.sh with the tag), after tools/gpu_r4_final.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_profiles.sh ${1:-r4} || exit 1
