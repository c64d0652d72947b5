# Usage: bash tools/gpu_pmc_gemm.sh <tag> <only> -- PMC passes over tools/gemm_bench.py for selected shapes
# (ring kernels on and off): HBM fetch, L2 hit/miss, SQ wait/busy counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pg}; ONLY=${2:-heads}
mkdir -p gpurun_out/pmcg_$TAG
rocprofv3 -L > gpurun_out/pmcg_$TAG/counters.txt 2>&1 || true
for RING in 0 1; do
  for PASS in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    N=$(echo $PASS | cut -d' ' -f1)
    SCD_GEMM_RING=$RING timeout -k 10 300 rocprofv3 --pmc $PASS --kernel-trace --output-format csv -d gpurun_out/pmcg_$TAG/r${RING}_$N -o run -- python3 tools/gemm_bench.py --only $ONLY --reps 3 > gpurun_out/pmcg_$TAG/r${RING}_$N.txt 2>&1 || exit 1
  done
done
ls gpurun_out/pmcg_$TAG
