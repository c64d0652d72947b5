# Round-6 calibration on one box:
#   1. tools/clock_probe.py: the bare bf16 MFMA peak on random data + in-kernel clocks of the step's big GEMMs
#      (stamped diagnostic build scdhip/libscdhip_stamp.so: make variant VAR=stamp VFLAGS=-DSCD_STAMP=1)
#   2. per-shape counters of the four big backward launches ALONE (tools/pmc_kernels.py cases): two SQ passes, FETCH_SIZE
#      and WRITE_SIZE, each pass its own rocprofv3 run
#   3. the same SQ passes IN THE STEP (Res10 bench), one row per (kernel, grid size)
# Outputs: gpurun_out/r6c_*.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 120 python3 tools/clock_probe.py > $O/r6c_clock.txt 2>&1 || { tail -5 $O/r6c_clock.txt; exit 1; }
SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_stamp.so timeout -k 10 120 python3 tools/clock_probe.py --gemms >> $O/r6c_clock.txt 2>&1 || { tail -5 $O/r6c_clock.txt; exit 1; }
grep -v amdgpu.ids $O/r6c_clock.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_ACTIVE_INST_LDS"
for c in heads_dgrad deconv3_dgrad wgrad_hm wgrad_d3; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/r6c_${c}_sq$i -o run -- python3 tools/pmc_kernels.py --case $c --reps 3 > $O/r6c_${c}_sq$i.log 2>&1 || { tail -5 $O/r6c_${c}_sq$i.log; exit 1; }
  done
  python3 tools/sq_summary.py --by-grid $O/r6c_${c}_sq1 $O/r6c_${c}_sq2 > $O/r6c_${c}_sq.txt || exit 1
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $k --output-format csv -d $O/r6c_${c}_$k -o run -- python3 tools/pmc_kernels.py --case $c --reps 3 > $O/r6c_${c}_$k.log 2>&1 || { tail -5 $O/r6c_${c}_$k.log; exit 1; }
  done
  f=$(find $O/r6c_${c}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  w=$(find $O/r6c_${c}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py $f $w $O/r6c_${c}_pmc.json > $O/r6c_${c}_hbm.txt || exit 1
  rm -rf $O/r6c_${c}_sq1 $O/r6c_${c}_sq2 $O/r6c_${c}_FETCH_SIZE $O/r6c_${c}_WRITE_SIZE
  echo "== $c"; cat $O/r6c_${c}_hbm.txt
done
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "conv_gemm_pp|conv_wgrad_pp2|heads384" --output-format csv -d $O/r6c_step_sq$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-calib > $O/r6c_step_sq$i.log 2>&1 || { tail -5 $O/r6c_step_sq$i.log; exit 1; }
done
python3 tools/sq_summary.py --by-grid $O/r6c_step_sq1 $O/r6c_step_sq2 > $O/r6c_step_sq.txt || exit 1
rm -rf $O/r6c_step_sq1 $O/r6c_step_sq2
echo calib done
