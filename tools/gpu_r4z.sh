# Usage: bash tools/gpu_r4z.sh -- the weight-gradient split reduce with its tail loads issued together (HEAD) vs the
# previous build (libscdhip_c1.so): the wgrad tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py -k "wgrad or deconv or reduce" > $O/r4z_tests.log 2>&1 || { tail -5 $O/r4z_tests.log; exit 1; }
tail -1 $O/r4z_tests.log
bash tools/gpu_abn.sh wr "SCD_X=0" "libscdhip_c1.so" || exit 1
grep "wgrad_reduce" $O/abn_wr_1_kernel_summary.txt $O/abn_wr_2_kernel_summary.txt
echo r4z done
