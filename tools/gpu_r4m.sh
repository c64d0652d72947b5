# Usage: bash tools/gpu_r4m.sh -- after removing the arrival flag's own LDS object (it made the compiler drain every
# LDS-DMA prefetch in the GEMM main loops) and templating the BN reduces on the fused tail: the GPU suite, then the
# round-3 HEAD (_r3/) against the current tree on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests > $O/r4m_tests.log 2>&1
rc=$?; tail -3 $O/r4m_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_r3ab.sh || exit 1
bash tools/gpu_abn.sh fin7 "SCD_BN_FIN_FUSE=0" "SCD_BN_FIN_FUSE=1" || exit 1
echo r4m done
