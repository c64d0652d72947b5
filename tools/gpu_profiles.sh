# Usage: bash tools/gpu_profiles.sh [tag] -- the round's measurement set, written to gpurun_out/<tag>_*:
#  PMC HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of the configs[3]/[4] dominant kernels (tools/pmc_kernels.py) and of
#  the Res10 bench command; then the bench lines (Res10 with the CPU baseline, Res50 1024^2 fp16, cornerNetCPool),
#  which read those PMC summaries, and rocprofv3 kernel traces of each bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5}
O=gpurun_out
mkdir -p $O
pmc() {   # pmc <name> <counter> <cmd...>
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${T}_pmc_${name}_$ctr -o run -- "$@" > $O/${T}_pmc_${name}_$ctr.log 2>&1 || return 1
  find $O/${T}_pmc_${name}_$ctr -name "*counter_collection.csv" | head -1
}
summ() {  # summ <name> <batch> <dtype> <command> <model> <S>
  local f w
  f=$(find $O/${T}_pmc_$1_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  w=$(find $O/${T}_pmc_$1_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $f $w $O/${T}_pmc_$1.json $2 $3 "$4" $5 $6 > $O/${T}_pmc_$1.txt && cp $O/${T}_pmc_$1.json profiles/
}
if [ -z "$SKIP_PMC" ]; then   # SKIP_PMC=1: the bench lines and traces only (the committed PMC summaries stay)
for c in FETCH_SIZE WRITE_SIZE; do
  pmc cornernet $c python3 tools/pmc_kernels.py --case lastconv,cpool_add || exit 1
  pmc res50_1024 $c python3 tools/pmc_kernels.py --case heads_res50 || exit 1
  pmc traffic $c python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-calib || exit 1
done
summ cornernet 32 bf16 "python3 tools/pmc_kernels.py --case lastconv,cpool_add" cornerNetCPool 512 || exit 1
summ res50_1024 16 fp16 "python3 tools/pmc_kernels.py --case heads_res50" centerOffsetRes50 1024 || exit 1
summ traffic 32 bf16 "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-calib" centerOffsetRes10 512 || exit 1
echo pmc done
fi
timeout -k 10 400 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cut -c1-200 $O/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-calib > $O/${T}_profbench.json 2> $O/${T}_prof.err || exit 1
python tools/prof_summary.py $O/${T}_prof/run_kernel_trace.csv $O/${T}_kernel_stats.csv > $O/${T}_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/${T}_prof/run_kernel_trace.csv > $O/${T}_step_timeline.txt 2>&1
timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --no-cpu-baseline --no-calib > $O/${T}_res50_1024_fp16_bench.json 2> $O/${T}_res50.err || exit 1
cut -c1-200 $O/${T}_res50_1024_fp16_bench.json
timeout -k 10 300 python bench.py --model cornerNetCPool --no-cpu-baseline --no-calib > $O/${T}_cornernet_bench.json 2> $O/${T}_corner.err || exit 1
cut -c1-200 $O/${T}_cornernet_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_res50 -o run -- python3 bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline --no-calib > $O/${T}_profbench_res50.json 2> $O/${T}_prof_res50.err || exit 1
python tools/prof_summary.py $O/${T}_prof_res50/run_kernel_trace.csv $O/${T}_res50_1024_fp16_kernel_stats.csv > $O/${T}_res50_1024_fp16_kernel_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_corner -o run -- python3 bench.py --model cornerNetCPool --steps 5 --warmup 2 --no-cpu-baseline --no-calib > $O/${T}_profbench_corner.json 2> $O/${T}_prof_corner.err || exit 1
python tools/prof_summary.py $O/${T}_prof_corner/run_kernel_trace.csv $O/${T}_cornernet_kernel_stats.csv > $O/${T}_cornernet_kernel_summary.txt 2>&1
echo all done
