# A/B of the heads tail backward launch knobs (SCD_HEADS_PXB pixels per block, SCD_HEADS_U unroll)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "2048 8" "1024 8" "512 8" "2048 4" "1024 4" "512 4" "4096 8"; do
  set -- $cfg
  SCD_HEADS_PXB=$1 SCD_HEADS_U=$2 timeout -k 10 120 python tools/hbm_bench.py > gpurun_out/hb_$1_$2.log 2>&1 || exit 1
  echo "PXB=$1 U=$2: $(grep heads_bwd gpurun_out/hb_$1_$2.log)"
done
