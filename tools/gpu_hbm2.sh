# Usage: bash tools/gpu_hbm2.sh <tag> "<cfg1>" "<cfg2>" ...  -- kernel tests, then the HBM bench under each env setting
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-h}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/hbm_bench.py --reps 20 > gpurun_out/hbm_$TAG.txt 2>&1 || exit 1
  grep "heads_bwd\|stem_pool" gpurun_out/hbm_$TAG.txt
done
