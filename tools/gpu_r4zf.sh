# Usage: bash tools/gpu_r4zf.sh -- the fp16 build's BN backward apply with two vectors in flight (HEAD) vs one
# (libscdhip_c3.so), on BASELINE configs[4] (centerOffsetRes50 1024² B=16 fp16): BN / model tests first, then bench
# lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py -k "bn or backward or Res50" > $O/r4zf_tests.log 2>&1 || { tail -5 $O/r4zf_tests.log; exit 1; }
tail -1 $O/r4zf_tests.log
BENCH_ARGS="--model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 10 --warmup 3" bash tools/gpu_abn.sh f16u "SCD_X=0" "libscdhip_c3.so" || exit 1
grep "bn_bwd_apply_kernel" $O/abn_f16u_1_kernel_summary.txt $O/abn_f16u_2_kernel_summary.txt
echo r4zf done
