# Usage: bash tools/gpu_r4_res50.sh [tag] -- BASELINE configs[4] only (centerOffsetRes50 1024² B=16 fp16): the bench
# line (PMC traffic from the committed profiles/<tag>_pmc_res50_1024.json) and its kernel trace, as
# tools/gpu_r3_profiles.sh writes them
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --no-cpu-baseline > $O/${T}_res50_1024_fp16_bench.json 2> $O/${T}_res50.err || exit 1
cut -c1-200 $O/${T}_res50_1024_fp16_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_res50 -o run -- python3 bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > $O/${T}_profbench_res50.json 2> $O/${T}_prof_res50.err || exit 1
python tools/prof_summary.py $O/${T}_prof_res50/run_kernel_trace.csv $O/${T}_res50_1024_fp16_kernel_stats.csv > $O/${T}_res50_1024_fp16_kernel_summary.txt 2>&1
rm -rf $O/${T}_prof_res50
echo res50 done
