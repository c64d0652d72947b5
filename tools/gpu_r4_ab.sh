# Usage: bash tools/gpu_r4_ab.sh -- round-4 set: the GPU suite + Res10 bench line + kernel trace (gpu_r4.sh r4a), then
# A/B of the committed-base library against this build and of the heads K-order switch (gpu_ab2.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4.sh r4a && bash tools/gpu_ab2.sh lib libscdhip_ab.so libscdhip.so && bash tools/gpu_ab2.sh serp SCD_HEADS_SERP=0 SCD_HEADS_SERP=1
