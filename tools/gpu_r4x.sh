# Usage: bash tools/gpu_r4x.sh -- branch-free loops (HEAD): the one-pass stem backward's column build / patch store,
# the BN backward apply and reduce specialised per mask kind, and the ping-pong GEMM epilogue's statistics by select
# and accumulate loads without a branch; against the stem + BN apply changes only (libscdhip_r4w.so) and the build
# before all of them (libscdhip_c0.so): the kernel / model GPU tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/r4x_tests.log 2>&1 || { tail -5 $O/r4x_tests.log; exit 1; }
tail -1 $O/r4x_tests.log
bash tools/gpu_abn.sh bf "SCD_X=0" "libscdhip_r4w.so" "libscdhip_c0.so" || exit 1
grep "conv_gemm_pp_kernel\|bn_bwd_reduce_kernel\|bn_bwd_apply_kernel\|stem_bwd_fused" $O/abn_bf_1_kernel_summary.txt $O/abn_bf_2_kernel_summary.txt $O/abn_bf_3_kernel_summary.txt
echo r4x done
