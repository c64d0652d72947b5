# Usage: bash tools/gpu_pmc_wgrad.sh <tag> <only> -- PMC passes over tools/wgrad_bench.py for one shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-w}; ONLY=${2:-layer1}
mkdir -p gpurun_out/pmcw_$TAG
N=0
for PASS in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE"; do
    N=$((N+1))
    timeout -s KILL 90 rocprofv3 --pmc $PASS --kernel-trace --output-format csv -d gpurun_out/pmcw_$TAG/p$N -o run -- python3 tools/wgrad_bench.py --only "$ONLY" --reps 2 > gpurun_out/pmcw_$TAG/p$N.txt 2>&1 || exit 1
done
python tools/pmc_table.py gpurun_out/pmcw_$TAG > gpurun_out/pmcw_$TAG/table.txt 2>&1
cat gpurun_out/pmcw_$TAG/table.txt
