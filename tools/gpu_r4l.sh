# Usage: bash tools/gpu_r4l.sh -- persistent stem conv kernels: stem / model GPU tests, then the A/B of the stem
# forward through y vs the pooled two-pass forward
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_parity_gpu.py > $O/r4l_tests.log 2>&1
rc=$?; tail -3 $O/r4l_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_abn.sh stem2 "SCD_STEM_POOLED=0" "SCD_STEM_POOLED=1" || exit 1
echo r4l done
