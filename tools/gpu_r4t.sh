# Usage: bash tools/gpu_r4t.sh -- the NQ 2 weight gradient with three stage buffers (HEAD) vs two
# (libscdhip_nb2.so): its parity / repeatability tests first, then bench lines and one kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py -k "wgrad or deconv" > $O/r4t_tests.log 2>&1 || { tail -5 $O/r4t_tests.log; exit 1; }
tail -1 $O/r4t_tests.log
bash tools/gpu_abn.sh nb3 "SCD_X=0" "libscdhip_nb2.so" || exit 1
grep "pp2_kernel<2>" $O/abn_nb3_1_kernel_summary.txt $O/abn_nb3_2_kernel_summary.txt
echo r4t done
