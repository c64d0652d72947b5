# Usage: bash tools/gpu_r4ze.sh -- the ring GEMM's shared epilogue without branch regions (BN-backward operand and
# accumulate loads from clamped addresses, statistics by select; HEAD) vs the previous build (libscdhip_c2.so): the
# kernel / model GPU tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/r4ze_tests.log 2>&1 || { tail -5 $O/r4ze_tests.log; exit 1; }
tail -1 $O/r4ze_tests.log
bash tools/gpu_abn.sh re "SCD_X=0" "libscdhip_c2.so" || exit 1
grep "ring_kernel\|conv_gemm_kernel" $O/abn_re_1_kernel_summary.txt $O/abn_re_2_kernel_summary.txt
echo r4ze done
