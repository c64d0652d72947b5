# Usage: bash tools/gpu_r4c.sh -- round-4 check set: the kernel / model tests touched this round, the direct-store
# epilogue A/B, the heads K-order PMC A/B, and the configs[4] Res50 1024^2 fp16 bench line with its kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf -s tests/test_kernels_gpu.py tests/test_model_gpu.py -k "serpentine or direct_store or l1p or bn_backward_sums or dgrad_with_bn or f9 or f11 or f3 or sgd or heads_fused" > $O/r4c_tests.log 2>&1
rc=$?; tail -3 $O/r4c_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_ab2.sh direct SCD_PP_DIRECT=0 SCD_PP_DIRECT=1 || exit 1
bash tools/gpu_pmc_ab.sh serp SCD_HEADS_SERP=0 SCD_HEADS_SERP=1 || exit 1
timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --no-cpu-baseline > $O/r4c_res50_1024_fp16_bench.json 2> $O/r4c_res50.err || exit 1
cut -c1-300 $O/r4c_res50_1024_fp16_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r4c_prof_res50 -o run -- python3 bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/r4c_prof_res50.err || exit 1
python tools/prof_summary.py $O/r4c_prof_res50/run_kernel_trace.csv $O/r4c_res50_1024_fp16_kernel_stats.csv > $O/r4c_res50_1024_fp16_kernel_summary.txt 2>&1
rm -rf $O/r4c_prof_res50
head -12 $O/r4c_res50_1024_fp16_kernel_summary.txt
echo r4c done
