# Usage: bash tools/gpu_diag.sh <tag> <only> -- ring GEMM ablations (SCD_GEMM_DEBUG 0/1/2) and PMC passes for selected shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dg}; ONLY=${2:-heads}
mkdir -p gpurun_out/diag_$TAG
for D in ${DBGS:-0 1 2}; do
  echo "== SCD_GEMM_DEBUG=$D"
  SCD_GEMM_DEBUG=$D timeout -k 10 120 python tools/gemm_bench.py --only $ONLY --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
done
for PASS in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr"; do
  N=$(echo $PASS | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-trace --output-format csv -d gpurun_out/diag_$TAG/$N -o run -- python3 tools/gemm_bench.py --only $ONLY --reps 3 > gpurun_out/diag_$TAG/$N.txt 2>&1 || exit 1
done
ls gpurun_out/diag_$TAG
