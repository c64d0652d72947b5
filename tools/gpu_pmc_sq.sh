# Usage: bash tools/gpu_pmc_sq.sh <tag> <kernel regex> -- SQ-block counters (two passes of at most 8 SQ + 2 GRBM
# counters each) of the kernels matching the regex in the Res10 bench command; per-kernel sums and per-launch means
# into gpurun_out/sq_<tag>.txt (tools/sq_summary.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; K=$2
O=gpurun_out
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$K" --output-format csv -d $O/sq_${T}_$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-calib > $O/sq_${T}_$i.log 2>&1 || { tail -5 $O/sq_${T}_$i.log; exit 1; }
done
python3 tools/sq_summary.py $O/sq_${T}_1 $O/sq_${T}_2 > $O/sq_${T}.txt || exit 1
cat $O/sq_${T}.txt
rm -rf $O/sq_${T}_1 $O/sq_${T}_2
