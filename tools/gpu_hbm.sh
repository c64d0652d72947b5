# Usage: bash tools/gpu_hbm.sh <tag>  -- GPU tests, HBM-kernel bench on the baseline library
# (scdhip/libscdhip_base.so) and the current one, GEMM bench with the split model off/on, step bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-h}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -f scd-resnet_amd/scdhip/libscdhip_base.so ]; then
  SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_base.so timeout -k 10 200 python tools/hbm_bench.py > gpurun_out/hbmA_$TAG.txt 2>&1 || exit 1
fi
timeout -k 10 200 python tools/hbm_bench.py > gpurun_out/hbmB_$TAG.txt 2>&1 || exit 1
paste gpurun_out/hbmA_$TAG.txt gpurun_out/hbmB_$TAG.txt 2>/dev/null | grep -v amdgpu.ids
SCD_WGRAD_NSMODEL=0 timeout -k 10 300 python tools/gemm_bench.py --reps 20 > gpurun_out/gemmA_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py --reps 20 > gpurun_out/gemmB_$TAG.txt 2>&1 || exit 1
paste gpurun_out/gemmA_$TAG.txt gpurun_out/gemmB_$TAG.txt | grep -v amdgpu.ids | grep "wgrad\|total"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json
exit $rc
