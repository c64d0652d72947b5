# Usage: bash tools/gpu_r4h.sh -- where the fused BN finalize's producer time goes: separate finalize vs fused with
# 4 / 8 replicas and the two timing-only ablations of the 4-replica build (no finalize arithmetic; no drain), then
# the host issue cost with the cached launch plans
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_model_gpu.py tests/test_kernels_gpu.py -k "fused_bn_finalize or f3 or f9 or wgrad or conv" > $O/r4h_tests.log 2>&1; rc=$?
tail -2 $O/r4h_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_abn.sh fin4 "SCD_BN_FIN_FUSE=0" "libscdhip_r4.so" "libscdhip_r8.so" "libscdhip_r4a1.so" "libscdhip_r4a2.so" || exit 1
timeout -k 10 300 python tools/host_overhead.py --steps 30 > $O/r4h_host_overhead.txt 2>&1 || exit 1
cat $O/r4h_host_overhead.txt
echo r4h done
