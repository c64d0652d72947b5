# Usage: bash tools/gpu_cpool.sh -- corner-pool parity tests and HBM timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corner_gpu.py tests/test_kernels_gpu.py -x -q -k "cpool or corner" --timeout 200 --timeout-method thread > gpurun_out/tests_cpool.log 2>&1; rc=$?
tail -5 gpurun_out/tests_cpool.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/hbm_bench.py --only cpool > gpurun_out/hbm_cpool.log 2>&1; rc=$?
cat gpurun_out/hbm_cpool.log
exit $rc
