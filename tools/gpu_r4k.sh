# Usage: bash tools/gpu_r4k.sh -- the GPU suite with the pooled stem forward (and the fused BN finalize off by default),
# then the A/B: stem forward through the full-resolution y vs the pooled two-pass forward
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests > $O/r4k_tests.log 2>&1
rc=$?; tail -3 $O/r4k_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_abn.sh stem "SCD_STEM_POOLED=0" "SCD_STEM_POOLED=1" || exit 1
echo r4k done
