# Usage: bash tools/gpu_r4g.sh -- fused-finalize parity tests on the replica-count variants, then the A/B: separate
# finalize vs fused with 16 / 4 / 1 statistics replicas
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for v in r4 r1; do
  SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_$v.so timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_model_gpu.py -k "fused_bn_finalize or f3 or f9 or full_size" > $O/r4g_tests_$v.log 2>&1 || { tail -5 $O/r4g_tests_$v.log; exit 1; }
  tail -1 $O/r4g_tests_$v.log
done
bash tools/gpu_abn.sh fin3 "SCD_BN_FIN_FUSE=0" "SCD_BN_FIN_FUSE=1" "libscdhip_r4.so SCD_BN_FIN_FUSE=1" "libscdhip_r1.so SCD_BN_FIN_FUSE=1" || exit 1
echo r4g done
