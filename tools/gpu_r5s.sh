# one-off (round 5): stream 1x1 GEMM tests, then Res50 1024^2 fp16 A/B: tiled kernels / stream kernel
export TMPDIR=/tmp; O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "stream" > $O/r5s_tests.log 2>&1; rc=$?; tail -3 $O/r5s_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 6 --warmup 2" bash tools/gpu_abn.sh s1x1 "SCD_GEMM_STREAM1X1=0" "SCD_GEMM_STREAM1X1=1" || exit 1
grep -E "conv1x1" $O/abn_s1x1_2_kernel_summary.txt
