# Usage: bash tools/gpu_r4u.sh -- the NQ 4 weight gradient with its G quarters issued at phases 0-1 (HEAD) vs 2-3
# (libscdhip_eg0.so): its parity / repeatability tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py -k "wgrad or deconv" > $O/r4u_tests.log 2>&1 || { tail -5 $O/r4u_tests.log; exit 1; }
tail -1 $O/r4u_tests.log
bash tools/gpu_abn.sh eg "SCD_X=0" "libscdhip_eg0.so" || exit 1
grep "pp2_kernel" $O/abn_eg_1_kernel_summary.txt $O/abn_eg_2_kernel_summary.txt
echo r4u done
