# Usage: bash tools/gpu_r4y.sh -- the batched weight pack with every group's loads issued before its stores (HEAD) vs
# the previous build (libscdhip_c1.so): kernel / model tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/r4y_tests.log 2>&1 || { tail -5 $O/r4y_tests.log; exit 1; }
tail -1 $O/r4y_tests.log
bash tools/gpu_abn.sh pk "SCD_X=0" "libscdhip_c1.so" || exit 1
grep "pack_weights" $O/abn_pk_1_kernel_summary.txt $O/abn_pk_2_kernel_summary.txt
echo r4y done
