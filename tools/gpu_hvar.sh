# Usage: bash tools/gpu_hvar.sh <tag> <variant libs...> -- heads rows of gemm_bench per variant library (timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
bash tools/gpu_variants.sh heads 20 "$@" > gpurun_out/var_$TAG.txt 2>&1 || { tail gpurun_out/var_$TAG.txt; exit 1; }
grep -E "==|fused" gpurun_out/var_$TAG.txt
