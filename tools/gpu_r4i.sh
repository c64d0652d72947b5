# Usage: bash tools/gpu_r4i.sh -- fused BN finalize with the register-resident descriptor tail: parity tests on the
# product build (16 replicas) and the 4-replica build, then separate vs fused with 16 / 8 / 4 replicas
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py > $O/r4i_tests.log 2>&1; rc=$?
tail -2 $O/r4i_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_r4.so timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_model_gpu.py -k "fused_bn_finalize or f3 or f9 or full_size" > $O/r4i_tests_r4.log 2>&1 || { tail -5 $O/r4i_tests_r4.log; exit 1; }
tail -1 $O/r4i_tests_r4.log
bash tools/gpu_abn.sh fin5 "SCD_BN_FIN_FUSE=0" "SCD_BN_FIN_FUSE=1" "libscdhip_r8.so" "libscdhip_r4.so" || exit 1
echo r4i done
