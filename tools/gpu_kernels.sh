set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/t_kernels.log 2>&1; rc=$?
tail -30 gpurun_out/t_kernels.log
exit $rc
