# Usage: bash tools/gpu_r4v.sh -- BN backward apply with two vectors in flight per thread (HEAD) vs one
# (libscdhip_au1.so): the BN / model tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py -k "bn or stem or backward" > $O/r4v_tests.log 2>&1 || { tail -5 $O/r4v_tests.log; exit 1; }
tail -1 $O/r4v_tests.log
bash tools/gpu_abn.sh au "SCD_X=0" "libscdhip_au1.so" || exit 1
grep "bn_bwd_apply_kernel" $O/abn_au_1_kernel_summary.txt $O/abn_au_2_kernel_summary.txt
echo r4v done
